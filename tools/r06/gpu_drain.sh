#!/bin/bash
# Round 6: the DMA GEMM loop with every LDS-DMA drained at every barrier (DRAIN, a diagnostic
# build) against the committed build: deviation counts under concurrency (race_probe.py stress).
set -o pipefail
for v in base DRAIN base DRAIN; do
  echo "== $v"
  ONEPOSE_LIB=$PWD/tools/ab/lib_$v.so RACE_N=40 timeout -k 10 400 python -u tools/r06/race_probe.py stress 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
done
