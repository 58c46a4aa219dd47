#!/bin/bash
# Matcher stream count on the final build: 2 (default) against 3, alternated, 20 and 300 steps.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05streams}
mkdir -p $O
line() {   # tag, args
  timeout -k 10 200 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'])"
}
for r in 1 2; do
  line s2_20_$r "--steps 20 --warmup 5"
  line s3_20_$r "--steps 20 --warmup 5 --match-streams 3"
  line s2_300_$r "--steps 300 --warmup 5"
  line s3_300_$r "--steps 300 --warmup 5 --match-streams 3"
  line s3p3_300_$r "--steps 300 --warmup 5 --match-streams 3 --pose-streams 3"
done
