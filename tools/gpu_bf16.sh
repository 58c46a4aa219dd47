#!/bin/bash
# bf16 attention mode: its GPU tests, then config 5 (2048 x 8192) and config 2 in bf16.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_matcher_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "bf16 or cache or prec" > gpurun_out/bf16_tests.log 2>&1 || { tail -30 gpurun_out/bf16_tests.log; exit 1; }
tail -2 gpurun_out/bf16_tests.log
timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --precision bf16 --n1 2048 --n3 8192 > gpurun_out/c5.json 2> gpurun_out/c5.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/c5.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c5 bf16', d['value'], r['avg_launch_us'], r['frac'], r['alone'], d['kernel_ms_per_step'])"
