#!/bin/bash
# Round-6 start: GPU suite, the driver's 20-step line (x2) and a 300-step line on the round-start
# build, the pose stage's phases (tools/pnp_probe) and the fp32 MLP conv 1 phases (phase_probe).
set -u
export TMPDIR=/tmp
O=gpurun_out/r06start
mkdir -p $O
timeout -k 10 60 ./tools/pnp_probe 900 0.1 > $O/pnp_probe_900.txt 2>&1 || { cat $O/pnp_probe_900.txt; exit 1; }
timeout -k 10 60 ./tools/pnp_probe 300 0.0 > $O/pnp_probe_300.txt 2>&1 || { cat $O/pnp_probe_300.txt; exit 1; }
cat $O/pnp_probe_900.txt
timeout -k 10 60 ./tools/phase_probe > $O/phase_probe.txt 2>&1 || { tail -30 $O/phase_probe.txt; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for i in 1 2; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_20_$i.json 2> $O/bench_20_$i.err || exit $?
python -c "import json; d=json.loads(open('$O/bench_20_$i.json').read().strip().splitlines()[-1]); print('20 steps', d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernel_ms_per_step'])"
done
timeout -k 10 200 python bench.py --gpus 1 --steps 300 --warmup 5 --no-cpu-baseline > $O/bench_300.json 2> $O/bench_300.err || exit $?
python -c "import json; d=json.loads(open('$O/bench_300.json').read().strip().splitlines()[-1]); print('300 steps', d['value'], d['ms_per_step'], d['roofline']['frac'])"
