#!/bin/bash
# Confirmation of the wide fp32 QKV default: the product (B) against tools/ab/lib_prev.so (A,
# 64 x 128 QKV): bits, GPU suite, three alternated pairs at 20 and 300 steps.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05qconf}
mkdir -p $O
A=$PWD/tools/ab/lib_prev.so
B=$PWD/onepose_amd/libonepose_hip.so
dump() { ONEPOSE_LIB=$2 timeout -k 10 300 python tools/bitcmp.py dump $O/$1.npz > $O/dump_$1.log 2>&1 || { tail -20 $O/dump_$1.log; rm -f $O/*.npz; exit 1; }; }
dump a $A
dump b $B
python tools/bitcmp.py cmp $O/a.npz $O/b.npz > $O/cmp.log 2>&1
echo "prev vs new: $(tail -1 $O/cmp.log)"
rm -f $O/*.npz
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
line() {   # tag, lib, args
  ONEPOSE_LIB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$1', d['value'], {x: k.get(x) for x in ('qkv_gemm','kv_reduce')})"
}
for r in 1 2 3; do
  line f20_A$r $A "--steps 20 --warmup 5"
  line f20_B$r $B "--steps 20 --warmup 5"
  line f300_A$r $A "--steps 300 --warmup 5"
  line f300_B$r $B "--steps 300 --warmup 5"
done
