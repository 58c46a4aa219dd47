#!/bin/bash
# Round 6: the single-process bench at 2 / 3 / 4 hardware queues per process (staged schedule).
set -o pipefail
O=gpurun_out/r06hwq2
mkdir -p $O
one() {   # name, env, args
  env $2 timeout -k 10 200 python bench.py --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || exit 1
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'])"
}
for i in 1 2; do
  for q in 2 3 4; do
    one s300_q${q}_$i "GPU_MAX_HW_QUEUES=$q" "--steps 300"
  done
done
