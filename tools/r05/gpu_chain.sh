#!/bin/bash
# Does the pose stage pace the matcher streams?  Default line against: no pose stage
# (diagnostic), 8 buffer slots, 4 pose streams, and the stage marks.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05chain}
mkdir -p $O
line() {   # tag, args
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 300 --warmup 5 $2 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d.get('stage_ms'))"
}
line base ""
line nopose "--diag-no-pose"
line slots8 "--slots 8"
line pose4 "--pose-streams 4 --slots 8"
line marks "--stage-marks"
line base2 ""
