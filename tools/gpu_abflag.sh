#!/bin/bash
# A/B of one bench flag on one box: bench.py alternately without (A) and with (B) FLAG.
#   FLAG="--unfused-pose" ROUNDS=3 STEPS=20 bash tools/gpu_abflag.sh
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in A B; do
    f=""; [ $v = B ] && f="$FLAG"
    timeout -k 10 200 python bench.py --steps ${STEPS:-200} --warmup 5 --no-cpu-baseline $f \
      ${BENCH_ARGS:-} > gpurun_out/abf_$v$r.json 2> gpurun_out/abf_$v$r.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/abf_$v$r.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
  done
done
