#!/bin/bash
# The driver's 20-step region under stage marks: where the fill / drain time goes.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-s20marks}
mkdir -p $O
run() {   # name, args
  timeout -k 10 200 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'], d.get('stage_ms'))"
}
run s20a "--steps 20 --warmup 5 --stage-marks"
run s20b "--steps 20 --warmup 5 --stage-marks"
run s20c "--steps 20 --warmup 5"
run s200 "--steps 200 --warmup 5 --stage-marks"
