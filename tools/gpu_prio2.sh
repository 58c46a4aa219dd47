#!/bin/bash
# Pose-stream priority, the driver's 20-step line: 6 alternating rounds of default vs high.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-prio2}
mkdir -p $O
run() {   # name, args
  timeout -k 10 200 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'])"
}
for i in 1 2 3 4 5 6; do
  run s20_p0_$i "--steps 20 --warmup 5"
  run s20_ph_$i "--steps 20 --warmup 5 --pose-priority -1"
done
