#!/bin/bash
# GPU test suite (optionally a subset: pass pytest args), then nothing else.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread "$@" > gpurun_out/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|differ|passed|failed" gpurun_out/gpu_tests.log | tail -60
exit $rc
