#!/bin/bash
# One call: the bit-identity check and same-box A/B of the last changes (gpu_r04_e.sh, two
# rounds), then the round's measurement set (gpu_r04_final.sh).  Stops at the first failure.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
ONEPOSE_LIB=$PWD/tools/ab/lib_base.so timeout -k 10 300 python tools/bitcmp.py dump $O/base.npz > $O/dump_base.log 2>&1 || { tail -20 $O/dump_base.log; exit 1; }
timeout -k 10 300 python tools/bitcmp.py dump $O/new.npz > $O/dump_new.log 2>&1 || { tail -20 $O/dump_new.log; exit 1; }
python tools/bitcmp.py cmp $O/base.npz $O/new.npz > $O/cmp.log 2>&1
rc=$?; tail -3 $O/cmp.log; rm -f $O/base.npz $O/new.npz
[ $rc -ne 0 ] && exit 1
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then lib=$PWD/tools/ab/lib_prev.so; else lib=""; fi
    ONEPOSE_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 300 --warmup 5 > $O/c2_$v$r.json 2> $O/c2_$v$r.err || exit $?
    python -c "import json; d=json.loads(open('$O/c2_$v$r.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('c2 $v$r', d['value'], d['roofline']['frac'], {x: k.get(x) for x in ('kv_reduce','score_gemm','mlp1_gemm','qkv_gemm')})"
  done
done
OUT=r04final bash tools/gpu_r04_final.sh
