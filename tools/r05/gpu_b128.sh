#!/bin/bash
# bf16 MLP conv 1 on the 8-wave 128 x 128 tile (tools/ab/lib_b128.so, B) against the product's
# 64 x 128 tile (A): bits, then same-box bf16 lines at config 2 and config 5.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05b128}
mkdir -p $O
A=$PWD/onepose_amd/libonepose_hip.so
B=$PWD/tools/ab/lib_b128.so
dump() { ONEPOSE_LIB=$2 timeout -k 10 300 python tools/bitcmp.py dump $O/$1.npz > $O/dump_$1.log 2>&1 || { tail -20 $O/dump_$1.log; rm -f $O/*.npz; exit 1; }; }
dump a $A
dump b $B
python tools/bitcmp.py cmp $O/a.npz $O/b.npz > $O/cmp.log 2>&1
echo "64x128 vs 128x128 bf16: $(tail -1 $O/cmp.log)"
rm -f $O/*.npz
line() {   # tag, lib, args
  ONEPOSE_LIB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; r=d['roofline']; print('$1', d['value'], r['avg_launch_us'], r['alone']['avg_launch_us'], r['frac'], {x: k.get(x) for x in ('mlp1_gemm','qkv_gemm','mlp2_gemm')})"
}
C5="--precision bf16 --desc-dtype fp16 --n1 2048 --n3 8192"
for r in 1 2; do
  line c5_A$r $A "--steps 100 --warmup 5 $C5"
  line c5_B$r $B "--steps 100 --warmup 5 $C5"
  line b2_A$r $A "--steps 300 --warmup 5 --precision bf16"
  line b2_B$r $B "--steps 300 --warmup 5 --precision bf16"
done
