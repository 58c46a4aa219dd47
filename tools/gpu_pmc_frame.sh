#!/bin/bash
# HBM traffic per kernel in the default two-stream graph schedule (vs tools/gpu_pmc.sh's serial
# eager pass): does sharing the chip with the other frame raise each kernel's HBM bytes?
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcf
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmcf/$c -o run -- \
    python3 bench.py --steps ${STEPS:-40} --warmup 5 --no-cpu-baseline \
    > gpurun_out/pmcf/bench_$c.json 2> gpurun_out/pmcf/bench_$c.err
  rc=$?
  echo "pmc $c rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_summary.py gpurun_out/pmcf > gpurun_out/pmcf/traffic.json
