#!/bin/bash
# Same-box A/B of two builds of the library: bits first (tools/bitcmp.py, 180 arrays), an
# optional GPU suite on B, then alternated bench lines.  Every round-5 variant A/B in DESIGN §8b
# ran in this shape (the variant built by tools/build_variant.sh with its -D flag):
#   A_LIB   build A (default tools/ab/lib_prev.so: the build before the change)
#   B_LIB   build B (default the product build)
#   LINES   which lines: any of f32 (20 / 300 steps, two pairs each), split, bf16, c5, c3
#           (default "f32 split c5")
#   PAIRS   pairs per fp32 line (default 2); TESTS=1 runs the GPU suite on B
#   KEYS    kernel_ms_per_step entries to print (default the layer GEMMs)
#   OUT     gpurun_out/ subdirectory (default r05ab); BITCMP_BIG=1 adds configs 5 / 3 to the bits
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05ab}
mkdir -p $O
A=${A_LIB:-$PWD/tools/ab/lib_prev.so}
B=${B_LIB:-$PWD/onepose_amd/libonepose_hip.so}
dump() { ONEPOSE_LIB=$2 timeout -k 10 300 python tools/bitcmp.py dump $O/$1.npz > $O/dump_$1.log 2>&1 || { tail -20 $O/dump_$1.log; rm -f $O/*.npz; exit 1; }; }
dump prev $A
dump new $B
python tools/bitcmp.py cmp $O/prev.npz $O/new.npz > $O/cmp.log 2>&1
echo "A vs B: $(tail -1 $O/cmp.log)"
rm -f $O/*.npz
if [ -n "${TESTS:-}" ]; then
  ONEPOSE_LIB=$B timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
fi
line() {   # tag, lib, args
  ONEPOSE_LIB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; r=d['roofline']; print('$1', d['value'], r['avg_launch_us'], r['alone']['avg_launch_us'], {x: k.get(x) for x in '${KEYS:-mlp1_gemm qkv_gemm mlp2_gemm score_gemm final_gemm}'.split()})"
}
C5="--precision bf16 --desc-dtype fp16 --n1 2048 --n3 8192"
for L in ${LINES:-f32 split c5}; do
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
