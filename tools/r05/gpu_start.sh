#!/bin/bash
# Round-5 start: MFMA order probe, GPU suite, the driver's 20-step line on the round-start build.
set -u
export TMPDIR=/tmp
O=gpurun_out/r05start
mkdir -p $O
timeout -k 10 60 ./tools/mfma_order > $O/mfma_order.txt 2>&1 || { cat $O/mfma_order.txt; exit 1; }
cat $O/mfma_order.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for i in 1 2; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_20_$i.json 2> $O/bench_20_$i.err || exit $?
python -c "import json; d=json.loads(open('$O/bench_20_$i.json').read().strip().splitlines()[-1]); print('20 steps', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
