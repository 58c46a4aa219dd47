#!/bin/bash
# End-of-session check of the committed build: GPU suite, default bench line (with the CPU
# baseline), the harness's 20-step line twice, and a rocprofv3 kernel-trace/stats pass.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-final}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
python -c "import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); print('default', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'))"
for i in 1 2; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_20_$i.json 2> $O/bench_20_$i.err || exit $?
python -c "import json; d=json.loads(open('$O/bench_20_$i.json').read().strip().splitlines()[-1]); print('20 steps', d['value'], d['ms_per_step'])"
done
mkdir -p $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline > $O/prof/bench.json 2> $O/prof/bench.err || exit $?
echo prof ok
