#!/bin/bash
# HBM traffic per kernel from PMC counters, per MI355X_MICROARCH.md's HBM section: FETCH_SIZE
# and WRITE_SIZE in separate passes (they do not fit one TCC pass), kernel-trace only.
# Summary (FETCH_SIZE x2 on gfx950 + WRITE_SIZE, per launch) -> gpurun_out/pmc/traffic.json
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc/$c -o run -- \
    python3 bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --serial --eager \
    > gpurun_out/pmc/bench_$c.json 2> gpurun_out/pmc/bench_$c.err
  rc=$?
  echo "pmc $c rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/traffic.json
