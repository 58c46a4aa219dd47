#!/bin/bash
# Config 5 (2048 x 8192, bf16 attention) counters on the final build: PMC FETCH_SIZE /
# WRITE_SIZE (separate passes), SQ counters, and a rocprofv3 kernel-trace/stats pass of the line.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04r
mkdir -p $O/pmc_c5 $O/sq_c5 $O/prof_c5
C5="--n1 2048 --n3 8192 --precision bf16"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_c5/$c -o run -- \
    python3 bench.py $C5 --steps 10 --warmup 3 --no-cpu-baseline --serial --eager \
    > $O/pmc_c5/bench_$c.json 2> $O/pmc_c5/bench_$c.err || exit $?
  echo "pmc $c ok"
done
python3 tools/pmc_summary.py $O/pmc_c5 > $O/pmc_c5/pmc_traffic.json || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $O/sq_c5/raw -o run -- \
  python3 bench.py $C5 --steps 10 --warmup 3 --no-cpu-baseline --serial --eager \
  > $O/sq_c5/bench.json 2> $O/sq_c5/bench.err || exit $?
python3 tools/pmc_summary.py --sq $O/sq_c5/raw > $O/sq_c5/sq_summary.json || exit $?
echo "sq ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- \
  python3 bench.py $C5 --steps 100 --warmup 5 --no-cpu-baseline > $O/prof_c5/bench.json 2> $O/prof_c5/bench.err || exit $?
echo "prof ok"
