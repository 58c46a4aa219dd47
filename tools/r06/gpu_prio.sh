#!/bin/bash
# Round 6: the staged schedule's pose streams (which now carry the final projection, score GEMM
# and winners) at high HIP stream priority vs the default (same box).
set -o pipefail
O=gpurun_out/r06prio
mkdir -p $O
one() {   # name, args
  timeout -k 10 200 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || exit 1
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'])"
}
for i in 1 2; do
  one s300_def_$i "--steps 300"
  one s300_hi_$i "--steps 300 --pose-priority -1"
  one s20_def_$i "--steps 20 --warmup 5"
  one s20_hi_$i "--steps 20 --warmup 5 --pose-priority -1"
done
