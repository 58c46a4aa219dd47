#!/bin/bash
# kv_fold with C's rows loaded in two round trips (buffer loads, scalar row offsets): bit-identity
# against tools/ab/lib_prev.so, the matcher GPU tests, same-box A/B against the previous commit
# (tools/ab/lib_head.so), config 2 fp32 (300 steps, two rounds) and config 5 bf16.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04m
mkdir -p $O
PREV=$PWD/tools/ab/lib_prev.so
HEAD=$PWD/tools/ab/lib_head.so
ONEPOSE_LIB=$PREV timeout -k 10 300 python tools/bitcmp.py dump $O/prev.npz > $O/dump_prev.log 2>&1 || { tail -20 $O/dump_prev.log; exit 1; }
timeout -k 10 300 python tools/bitcmp.py dump $O/new.npz > $O/dump_new.log 2>&1 || { tail -20 $O/dump_new.log; exit 1; }
python tools/bitcmp.py cmp $O/prev.npz $O/new.npz > $O/cmp.log 2>&1
rc=$?; tail -2 $O/cmp.log; rm -f $O/*.npz
[ $rc -ne 0 ] && exit 1
timeout -k 10 400 python -u -m pytest tests/test_matcher_gpu.py tests/test_configs_gpu.py -m gpu -x -q -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
line() {   # tag, lib, args
  ONEPOSE_LIB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$1', d['value'], {x: k.get(x) for x in ('kv_reduce','conf','mlp1_gemm')})"
}
for r in 1 2; do
  line c2_A$r $HEAD "--steps 300 --warmup 5"
  line c2_B$r "" "--steps 300 --warmup 5"
done
line c5_A $HEAD "--n1 2048 --n3 8192 --precision bf16 --steps 100 --warmup 3"
line c5_B "" "--n1 2048 --n3 8192 --precision bf16 --steps 100 --warmup 3"
