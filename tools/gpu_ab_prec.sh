#!/bin/bash
# A/B of the matcher precision modes on one box: GPU matcher tests of the bf16 modes, then the
# config-2 bench (300 steps) in fp32 / fp32_split, alternating, and config 5 in bf16.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_matcher_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "split or bf16 or fixture or cache or tables" > gpurun_out/prec_tests.log 2>&1 || { tail -30 gpurun_out/prec_tests.log; exit 1; }
tail -2 gpurun_out/prec_tests.log
for r in 1 2; do
  for p in fp32 fp32_split; do
    timeout -k 10 200 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --precision $p > gpurun_out/ab_$p.json 2> gpurun_out/ab_$p.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/ab_$p.json').read().strip().splitlines()[-1]); print('$p', d['value'], d['roofline']['avg_launch_us'], d['kernel_ms_per_step'])"
  done
done
timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --precision bf16 --n1 2048 --n3 8192 > gpurun_out/ab_c5.json 2> gpurun_out/ab_c5.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/ab_c5.json').read().strip().splitlines()[-1]); print('c5 bf16', d['value'], d['roofline'], d['kernel_ms_per_step'])"
