#!/bin/bash
# Configs 3 (reference fixture) and 4 (numpy oracle) through the cached path, fp32 and split.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04t
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_configs_gpu.py -m gpu -k "config3 or config4" -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/tests.log | tail -4
