#!/bin/bash
# The fp32 QKV on 16-deep stages (tools/ab/lib_qk16.so, B) against the
# product's 32-deep 64 x 128 QKV tile (A): bits, the GPU suite on B, same-box fp32 lines.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05qk16}
mkdir -p $O
A=$PWD/onepose_amd/libonepose_hip.so
B=$PWD/tools/ab/lib_qk16.so
dump() { ONEPOSE_LIB=$2 timeout -k 10 300 python tools/bitcmp.py dump $O/$1.npz > $O/dump_$1.log 2>&1 || { tail -20 $O/dump_$1.log; rm -f $O/*.npz; exit 1; }; }
dump a $A
dump b $B
python tools/bitcmp.py cmp $O/a.npz $O/b.npz > $O/cmp.log 2>&1
echo "QKV 32-deep vs 16-deep: $(tail -1 $O/cmp.log)"
rm -f $O/*.npz
if [ -n "${TESTS:-}" ]; then
  ONEPOSE_LIB=$B timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
fi
line() {   # tag, lib, args
  ONEPOSE_LIB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; r=d['roofline']; print('$1', d['value'], r['avg_launch_us'], r['alone']['avg_launch_us'], {x: k.get(x) for x in ('mlp1_gemm','qkv_gemm','mlp2_gemm')})"
}
for r in 1 2; do
  line sp20_A$r $A "--steps 20 --warmup 5 --precision fp32"
  line sp20_B$r $B "--steps 20 --warmup 5 --precision fp32"
  line sp300_A$r $A "--steps 300 --warmup 5 --precision fp32"
  line sp300_B$r $B "--steps 300 --warmup 5 --precision fp32"
done
