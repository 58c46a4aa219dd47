#!/bin/bash
# Same-box A/B of the product build (B) against tools/ab/lib_prev.so (A, the build before the
# change): bits first (tools/bitcmp.py), optional GPU suite, then alternated bench lines.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05ab}
mkdir -p $O
A=$PWD/tools/ab/lib_prev.so
B=$PWD/onepose_amd/libonepose_hip.so
dump() { ONEPOSE_LIB=$2 timeout -k 10 300 python tools/bitcmp.py dump $O/$1.npz > $O/dump_$1.log 2>&1 || { tail -20 $O/dump_$1.log; rm -f $O/*.npz; exit 1; }; }
dump prev $A
dump new $B
python tools/bitcmp.py cmp $O/prev.npz $O/new.npz > $O/cmp.log 2>&1
echo "prev vs new: $(tail -1 $O/cmp.log)"
rm -f $O/*.npz
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
fi
line() {   # tag, lib, args
  ONEPOSE_LIB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; r=d['roofline']; print('$1', d['value'], r['avg_launch_us'], r['alone']['avg_launch_us'], {x: k.get(x) for x in ('mlp1_gemm','qkv_gemm','mlp2_gemm','score_gemm','final_gemm')})"
}
for r in 1 2; do
  line n20_A$r $A "--steps 20 --warmup 5"
  line n20_B$r $B "--steps 20 --warmup 5"
  line n300_A$r $A "--steps 300 --warmup 5"
  line n300_B$r $B "--steps 300 --warmup 5"
done
line sp_A $A "--steps 300 --warmup 5 --precision fp32_split"
line sp_B $B "--steps 300 --warmup 5 --precision fp32_split"
line c5_A $A "--steps 100 --warmup 5 --precision bf16 --desc-dtype fp16 --n1 2048 --n3 8192"
line c5_B $B "--steps 100 --warmup 5 --precision bf16 --desc-dtype fp16 --n1 2048 --n3 8192"
