#!/bin/bash
# One pose stream against two (default), alternated, 20 and 300 steps.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05posestreams}
mkdir -p $O
line() {   # tag, args
  timeout -k 10 200 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'])"
}
for r in 1 2 3; do
  line p2_20_$r "--steps 20 --warmup 5"
  line p1_20_$r "--steps 20 --warmup 5 --pose-streams 1"
done
for r in 1 2; do
  line p2_300_$r "--steps 300 --warmup 5"
  line p1_300_$r "--steps 300 --warmup 5 --pose-streams 1"
done
