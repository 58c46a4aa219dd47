#!/bin/bash
# Round-4 start: GPU suite + the driver's 20-step line + a 300-step line on the round-start build.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04_start}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_20.json 2> $O/bench_20.err || exit $?
timeout -k 10 300 python bench.py --gpus 1 --steps 300 --warmup 5 --no-cpu-baseline > $O/bench_300.json 2> $O/bench_300.err || exit $?
python -c "
import json
for n in ('20','300'):
    d=json.loads(open('$O/bench_'+n+'.json').read().strip().splitlines()[-1]); print(n, d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('kernel_ms_per_step'))"
