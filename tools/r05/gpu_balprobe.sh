#!/bin/bash
# Where the balanced MLP conv 1 kernel's time goes: the same launch with its global loads, its
# MFMAs or its LDS stores left out (tools/bal_probe.hip built with BAL_PROBE_* knobs).
set -u
O=gpurun_out/r05balprobe
mkdir -p $O
for v in "" _EPI_TILE; do
  timeout -k 10 120 ./tools/bal_probe$v > $O/probe$v.txt 2>&1 || { cat $O/probe$v.txt; exit 1; }
  echo "== bal_probe$v"; grep -B3 "M 1024/4096 B 1 acc0 0/0" $O/probe$v.txt | grep "us mean"
done
