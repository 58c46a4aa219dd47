#!/bin/bash
# Tile sweep of the big SuperPoint conv layers: rocprof per variant (measurement only).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
for v in ${VARIANTS:-0 1 2 3 5 6}; do
  rm -rf gpurun_out/sweep/v$v
  ONEPOSE_SP_TILE=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sweep/v$v -o t -- python3 tools/sp_bench.py --batch 1 8 --iters 10 > gpurun_out/sweep/v$v.log 2>&1 || exit $?
  echo "variant $v"; grep batch gpurun_out/sweep/v$v.log
done
