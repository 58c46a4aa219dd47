#!/bin/bash
# A/B frames/s on one box: bench.py alternately with the current library (B) and
# tools/ab/lib_base.so (A, built from an older commit), ROUNDS times each.
#   ROUNDS=3 BENCH_ARGS="--steps 200" bash tools/ab.sh
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-3}
for r in $(seq 1 $ROUNDS); do
  for v in A B; do
    if [ $v = A ]; then lib=$PWD/tools/ab/lib_base.so; else lib=""; fi
    ONEPOSE_LIB=$lib timeout -k 10 200 python bench.py --steps ${STEPS:-200} --warmup 5 \
      --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$v$r.json 2> gpurun_out/ab_$v$r.err || exit $?
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v$r.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_us'], {k: v for k, v in list(d.get('kernel_ms_per_step', {}).items())[:6]})"
  done
done
