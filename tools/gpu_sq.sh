#!/bin/bash
# MFMA-busy and wave-state SQ counters per kernel over a short bench run (one rocprofv3 --pmc
# pass, kernel-trace only; 7 SQ + 1 GRBM counters fit one pass on gfx950).
# Summary -> gpurun_out/sq/sq_summary.json (tools/pmc_summary.py --sq).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/sq
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d gpurun_out/sq/raw -o run -- \
  python3 bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --serial --eager ${BENCH_ARGS:-} \
  > gpurun_out/sq/bench.json 2> gpurun_out/sq/bench.err
rc=$?
echo "sq rc=$rc"
[ $rc -ne 0 ] && exit $rc
python3 tools/pmc_summary.py --sq gpurun_out/sq/raw > gpurun_out/sq/sq_summary.json
