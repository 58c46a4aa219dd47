#!/bin/bash
# Two vs three concurrent matcher streams at config 2 (fp32), alternating.
set -u
export TMPDIR=/tmp
O=gpurun_out/streams3
mkdir -p $O
run() {   # name, args
  timeout -k 10 200 python bench.py --steps 300 --warmup 5 --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['roofline']['avg_launch_us'])"
}
run s2a "--match-streams 2"
run s3a "--match-streams 3"
run s2b "--match-streams 2"
run s3b "--match-streams 3"
run s4a "--match-streams 4"
