#!/bin/bash
# bf16 MLP conv 1 on the 256 x 128 DMA-3 tile: probe (bits + alone timing + phases), whole-library
# bit comparison against the 64 x 128 build (the product build) and round 4, optional GPU
# suite, then same-box bf16 lines (config 2 and config 5) A = product (64 x 128), B = tools/ab/lib_ws.so.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05wsab}
mkdir -p $O
A=$PWD/onepose_amd/libonepose_hip.so
B=$PWD/tools/ab/lib_ws.so
R04=$PWD/tools/ab/lib_r04.so
timeout -k 10 120 ./tools/ws_probe > $O/ws_probe.txt 2>&1 || { cat $O/ws_probe.txt; exit 1; }
grep -A2 timed $O/ws_probe.txt; tail -1 $O/ws_probe.txt
if [ -z "${NOPHASE:-}" ]; then
timeout -k 10 180 ./tools/phase_probe ws > $O/phase_ws.txt 2>&1 || { tail -5 $O/phase_ws.txt; exit 1; }
grep -B1 "^bf16" $O/phase_ws.txt | tail -12
fi
dump() { ONEPOSE_LIB=$2 timeout -k 10 300 python tools/bitcmp.py dump $O/$1.npz > $O/dump_$1.log 2>&1 || { tail -20 $O/dump_$1.log; rm -f $O/*.npz; exit 1; }; }
dump m64 $A
dump ws $B
dump r04 $R04
for pair in "m64 ws" "r04 ws"; do
  set -- $pair
  python tools/bitcmp.py cmp $O/$1.npz $O/$2.npz > $O/cmp_$1_$2.log 2>&1
  echo "$1 vs $2: $(tail -1 $O/cmp_$1_$2.log)"
done
rm -f $O/*.npz
if [ -n "${TESTS:-}" ]; then
  ONEPOSE_LIB=$B timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
fi
line() {   # tag, lib, args
  ONEPOSE_LIB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; r=d['roofline']; print('$1', d['value'], r['kernel'], r['avg_launch_us'], r['frac'], r['alone']['avg_launch_us'], {x: k.get(x) for x in ('mlp1_gemm','qkv_gemm','mlp2_gemm')})"
}
C5="--precision bf16 --desc-dtype fp16 --n1 2048 --n3 8192"
for r in 1 2; do
  line c5_A$r $A "--steps 100 --warmup 5 $C5"
  line c5_B$r $B "--steps 100 --warmup 5 $C5"
  line b2_A$r $A "--steps 200 --warmup 5 --precision bf16"
  line b2_B$r $B "--steps 200 --warmup 5 --precision bf16"
done
