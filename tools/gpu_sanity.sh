#!/bin/bash
# Sanity pass on a fresh box: GPU suite, then the harness's 20-step bench line.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-sanity}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for i in 1 2; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_20_$i.json 2> $O/bench_20_$i.err || exit $?
python -c "import json; d=json.loads(open('$O/bench_20_$i.json').read().strip().splitlines()[-1]); print('20 steps', d['value'], d['ms_per_step'], d['kernel_ms_per_step'])"
done
timeout -k 10 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline > $O/bench_300.json 2> $O/bench_300.err || exit $?
python -c "import json; d=json.loads(open('$O/bench_300.json').read().strip().splitlines()[-1]); print('300 steps', d['value'], d['ms_per_step'], d['kernel_ms_per_step'])"
