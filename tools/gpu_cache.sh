#!/bin/bash
# Object-cache check: matcher / pipeline / inference / sharded GPU tests, then the headline
# bench with and without the per-object prefix cache.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_matcher_gpu.py tests/test_pipeline_gpu.py \
  tests/test_inference_gpu.py tests/test_sharded_gpu.py -q -x -rf --timeout=300 \
  > gpurun_out/cache_tests.log 2>&1 || { tail -40 gpurun_out/cache_tests.log; exit 1; }
tail -3 gpurun_out/cache_tests.log
for mode in cache nocache; do
  flag=""; [ $mode = nocache ] && flag="--no-object-cache"
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 20 $flag \
    > gpurun_out/bench_$mode.json 2> gpurun_out/bench_$mode.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/bench_$mode.json').read().strip().splitlines()[-1]); print('$mode', d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'], d['frame_roofline'], d['pose'])"
done
