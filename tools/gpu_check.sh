#!/bin/bash
# One GPU-box round: GPU tests, smoke, then a short bench.  Each step has its own time
# limit; nothing further runs after a crash (exit status other than 0/1 from pytest).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-30}
timeout -k 10 ${TEST_TIMEOUT:-600} python -m pytest tests -m gpu -q -rf --timeout=400 ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps $STEPS --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
exit $rc
