#!/bin/bash
# A/B of an environment setting on one box, alternating:  VAR=NAME A=val B=val bash tools/gpu_envab.sh
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in A B; do
    if [ $v = A ]; then val=$A; else val=$B; fi
    env $VAR=$val timeout -k 10 200 python bench.py --steps ${STEPS:-300} --warmup ${WARM:-10} --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/env_$v.json 2> gpurun_out/env_$v.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/env_$v.json').read().strip().splitlines()[-1]); print('$v', '$val', d['value'], d['roofline']['avg_launch_us'], d.get('stage_ms',''))"
  done
done
