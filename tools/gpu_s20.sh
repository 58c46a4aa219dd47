#!/bin/bash
# Dev probe: the harness's 20-step region after W warm-up steps (W sweep, interleaved rounds)
export TMPDIR=/tmp; mkdir -p gpurun_out
run() { timeout -k 10 200 python bench.py --steps ${STEPS:-20} --no-cpu-baseline "$@" > gpurun_out/v.json 2>/dev/null || exit 1; python -c "import json;d=json.loads(open('gpurun_out/v.json').read().strip().splitlines()[-1]);print('$*', d['value'], d['ms_per_step'])"; }
for r in 1 2 3; do for w in ${WS:-5 20 50 100 200}; do run --warmup $w; done; done
