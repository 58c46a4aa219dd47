#!/bin/bash
# Round 6, last check of the committed build: GPU suite, smoke(), the default bench line and the
# driver's 20-step line twice.
set -u
O=gpurun_out/r06end
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
python -c "import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); print('default', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'))"
for i in 1 2; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_20_$i.json 2> $O/bench_20_$i.err || exit $?
python -c "import json; d=json.loads(open('$O/bench_20_$i.json').read().strip().splitlines()[-1]); print('20 steps', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
