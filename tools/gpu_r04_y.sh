#!/bin/bash
# The phase probe's wide-tile cases again, after the DMA loop's scheduling fix.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04y
mkdir -p $O
timeout -k 10 180 ./tools/phase_probe big > $O/phase_big.txt 2>&1 || { tail -5 $O/phase_big.txt; exit 1; }
grep -v "^ *phases" $O/phase_big.txt | cut -c1-110
