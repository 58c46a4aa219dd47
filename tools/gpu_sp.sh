#!/bin/bash
# SuperPoint on one GPU box: parity tests, timing, and a rocprofv3 kernel summary.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/spprof
timeout -k 10 400 python -m pytest tests/test_superpoint_gpu.py -q -rf -x --timeout=300 > gpurun_out/sp_tests.log 2>&1
rc=$?
tail -15 gpurun_out/sp_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/sp_bench.py --iters 30 > gpurun_out/sp_bench.log 2>&1 || exit $?
grep batch gpurun_out/sp_bench.log
rm -rf gpurun_out/spprof/*
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/spprof -o sp -- python3 tools/sp_bench.py --batch 1 --iters 20 > gpurun_out/spprof/log.txt 2>&1 || exit $?
exit $rc
