#!/bin/bash
# Round-3 measurement set, part B: PMC HBM traffic (FETCH_SIZE and WRITE_SIZE in separate
# passes, MI355X_MICROARCH.md HBM section) and SQ MFMA-busy counters, for config 2 (fp32) and
# config 5 (bf16 attention).  Each pass is its own rocprofv3 run with --kernel-trace only.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r03}
for cfg in c2 c5; do
  if [ $cfg = c5 ]; then ARGS="--precision bf16 --n1 2048 --n3 8192"; else ARGS=""; fi
  mkdir -p $O/pmc_$cfg
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_$cfg/$c -o run -- \
      python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --serial --eager $ARGS \
      > $O/pmc_$cfg/bench_$c.json 2> $O/pmc_$cfg/bench_$c.err || exit $?
    echo "pmc $cfg $c ok"
  done
  python3 tools/pmc_summary.py $O/pmc_$cfg > $O/pmc_$cfg/traffic.json || exit $?
  mkdir -p $O/sq_$cfg
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d $O/sq_$cfg/raw -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --serial --eager $ARGS \
    > $O/sq_$cfg/bench.json 2> $O/sq_$cfg/bench.err || exit $?
  python3 tools/pmc_summary.py --sq $O/sq_$cfg/raw > $O/sq_$cfg/sq_summary.json || exit $?
  echo "sq $cfg ok"
done
