#!/bin/bash
# The whole GPU suite on the final tree.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04u
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
