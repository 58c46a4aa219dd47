#!/bin/bash
# QKV on the 8-wave 128 x 128 stand-in tile (64-row KV chunks, the same bits): fp32
# (tools/ab/lib_qw.so) and split (tools/ab/lib_qws.so) against the product (A).
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05qwide}
mkdir -p $O
A=$PWD/onepose_amd/libonepose_hip.so
B1=$PWD/tools/ab/lib_qw.so
B2=$PWD/tools/ab/lib_qws.so
dump() { ONEPOSE_LIB=$2 timeout -k 10 300 python tools/bitcmp.py dump $O/$1.npz > $O/dump_$1.log 2>&1 || { tail -20 $O/dump_$1.log; rm -f $O/*.npz; exit 1; }; }
dump a $A
dump qw $B1
dump qws $B2
for v in qw qws; do
  python tools/bitcmp.py cmp $O/a.npz $O/$v.npz > $O/cmp_$v.log 2>&1
  echo "product vs $v: $(tail -1 $O/cmp_$v.log)"
done
rm -f $O/*.npz
line() {   # tag, lib, args
  ONEPOSE_LIB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; r=d['roofline']; print('$1', d['value'], r['avg_launch_us'], {x: k.get(x) for x in ('mlp1_gemm','qkv_gemm','mlp2_gemm','kv_reduce')})"
}
for r in 1 2; do
  line f20_A$r $A "--steps 20 --warmup 5"
  line f20_B$r $B1 "--steps 20 --warmup 5"
  line f300_A$r $A "--steps 300 --warmup 5"
  line f300_B$r $B1 "--steps 300 --warmup 5"
  line sp_A$r $A "--steps 300 --warmup 5 --precision fp32_split"
  line sp_B$r $B2 "--steps 300 --warmup 5 --precision fp32_split"
done
