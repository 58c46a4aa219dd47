#!/bin/bash
# Round-end style check: every GPU test, smoke(), then the default bench line.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf --timeout=400 > gpurun_out/gpu_all.log 2>&1
rc=$?
tail -6 gpurun_out/gpu_all.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 3; }
cat gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench_default.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline'], d.get('cpu_baseline'))"
exit $rc
