#!/bin/bash
# Core clock while the default bench runs (tools/clock_sampler in a second process).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps ${STEPS:-6000} --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/clk_bench.json 2> gpurun_out/clk_bench.err &
bp=$!
sleep ${DELAY:-25}
timeout -k 5 60 ./tools/clock_sampler 150
wait $bp
python -c "import json; d=json.loads(open('gpurun_out/clk_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
