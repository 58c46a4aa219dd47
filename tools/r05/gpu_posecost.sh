#!/bin/bash
# What the pose stage costs the driver-shaped 20-step line: default against --diag-no-pose
# (diagnostic: matchers only), alternated, plus the stage marks of one default run.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05posecost}
mkdir -p $O
line() {   # tag, args
  timeout -k 10 200 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d.get('stage_ms'))"
}
for r in 1 2 3; do
  line p20_$r "--steps 20 --warmup 5"
  line np20_$r "--steps 20 --warmup 5 --diag-no-pose"
done
line marks20 "--steps 20 --warmup 5 --stage-marks"
