#!/bin/bash
# One bench line per argument set (VARIANTS, ';'-separated), ROUNDS rounds, same box.
#   VARIANTS="--match-streams 2;--match-streams 3" bash tools/gpu_variants.sh
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
IFS=';' read -ra VS <<< "${VARIANTS}"
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for v in "${VS[@]}"; do
    i=$((i+1))
    timeout -k 10 200 python bench.py --steps ${STEPS:-200} --warmup 5 --no-cpu-baseline $v \
      > gpurun_out/var_$i.json 2> gpurun_out/var_$i.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/var_$i.json').read().strip().splitlines()[-1]); print('[$v]', d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_us'], list(d['kernel_ms_per_step'].items())[:4])"
  done
done
