#!/bin/bash
# fp32 MLP conv 2 tile shapes in the phase probe (production 64 x 32 K-split vs 8-wave tiles).
set -u
export TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 180 ./tools/phase_probe mlp2 > $O/phase_mlp2.txt 2>&1 || { tail -5 $O/phase_mlp2.txt; exit 1; }
cut -c1-200 $O/phase_mlp2.txt
