#!/bin/bash
# One call: the 256 x 128 tile A/B (tools/r05/gpu_wsab.sh, GPU suite on that build), then the
# drop-in entry's throughput with the resident object (tools/entry_bench.py).
set -u
export TMPDIR=/tmp
TESTS=1 OUT=r05b ./tools/r05/gpu_wsab.sh || exit $?
O=gpurun_out/r05b
timeout -k 10 600 python -u tools/entry_bench.py --frames 64 --n3 4096 --out $O/entry.json > $O/entry.log 2>&1 || { tail -30 $O/entry.log; exit 1; }
grep -E "^(superpoint|detections)" $O/entry.log
