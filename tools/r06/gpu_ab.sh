#!/bin/bash
# Round-6 same-box A/B: bits over the tools/bitcmp.py arrays (BITCMP_BIG=1: 270), the GPU
# suite on B (TESTS=1), then alternated bench lines (LINES: f32 = 20 + 300 steps, PAIRS pairs;
# split, bf16, c5, c3 one pair each).  A = the round-5 build (tools/ab/lib_r05.so) by default.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06ab}
mkdir -p $O
A=${A_LIB:-$PWD/tools/ab/lib_r05.so}
B=${B_LIB:-$PWD/onepose_amd/libonepose_hip.so}
if [ -z "${NOBITS:-}" ]; then
  dump() { ONEPOSE_LIB=$2 BITCMP_BIG=${BITCMP_BIG:-1} timeout -k 10 300 python tools/bitcmp.py dump $O/$1.npz > $O/dump_$1.log 2>&1 || { tail -20 $O/dump_$1.log; rm -f $O/*.npz; exit 1; }; }
  dump prev $A
  dump new $B
  python tools/bitcmp.py cmp $O/prev.npz $O/new.npz > $O/cmp.log 2>&1
  echo "A vs B: $(tail -1 $O/cmp.log)"
  rm -f $O/*.npz
fi
if [ -n "${TESTS:-}" ]; then
  ONEPOSE_LIB=$B timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
fi
line() {   # tag, lib, args
  ONEPOSE_LIB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; r=d['roofline']; print('$1', d['value'], r['avg_launch_us'], {x: k.get(x) for x in '${KEYS:-mlp1_gemm qkv_gemm mlp2_gemm pnp_ransac pnp_refit kv_reduce}'.split()})"
}
C5="--precision bf16 --desc-dtype fp16 --n1 2048 --n3 8192"
for L in ${LINES:-f32}; do
  case $L in
    f32)
      for r in $(seq 1 ${PAIRS:-2}); do
        line n20_A$r $A "--steps 20 --warmup 5"
        line n20_B$r $B "--steps 20 --warmup 5"
        line n300_A$r $A "--steps 300 --warmup 5"
        line n300_B$r $B "--steps 300 --warmup 5"
      done ;;
    split)
      line sp_A $A "--steps 300 --warmup 5 --precision fp32_split"
      line sp_B $B "--steps 300 --warmup 5 --precision fp32_split" ;;
    bf16)
      line bf_A $A "--steps 300 --warmup 5 --precision bf16"
      line bf_B $B "--steps 300 --warmup 5 --precision bf16" ;;
    c5)
      line c5_A $A "--steps 100 --warmup 5 $C5"
      line c5_B $B "--steps 100 --warmup 5 $C5" ;;
    c3)
      line c3_A $A "--n3 16384 --batch 32 --steps 10 --warmup 2"
      line c3_B $B "--n3 16384 --batch 32 --steps 10 --warmup 2" ;;
  esac
done
