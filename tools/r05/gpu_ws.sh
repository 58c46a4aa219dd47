#!/bin/bash
# The 256 x 128 eight-wave bf16 MLP conv 1 tile against the 64 x 128 tile: bit comparison + timing,
# then the phase probe's per-phase cycles for both.
set -u
O=gpurun_out/r05ws
mkdir -p $O
timeout -k 10 120 ./tools/ws_probe > $O/ws_probe.txt 2>&1 || { cat $O/ws_probe.txt; exit 1; }
tail -14 $O/ws_probe.txt
timeout -k 10 180 ./tools/phase_probe ws > $O/phase_ws.txt 2>&1; rc=$?
cat $O/phase_ws.txt
exit $rc
