#!/bin/bash
# Generates the phase probes' copies of the production sources: every "// @phase N" marker in
# gemm.hip / pnp.hip becomes a stamp macro the probe defines (ONEPOSE_GEMM_PHASE /
# ONEPOSE_PNP_PHASE). The library itself has no hooks. Then builds the two probes:
#   bash tools/probe_src.sh && ./tools/phase_probe && ./tools/pnp_probe
set -eu
cd "$(dirname "$0")/.."
mkdir -p tools/_gen
sed -E 's#// @phase ([0-9]+)#ONEPOSE_GEMM_PHASE(\1);#' onepose_amd/csrc/gemm.hip > tools/_gen/gemm.hip
sed -E 's#// @phase ([0-9]+)#ONEPOSE_PNP_PHASE(\1);#' onepose_amd/csrc/pnp.hip > tools/_gen/pnp.hip
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
$HIPCC --offload-arch=gfx950 -O3 -std=c++17 -w -Ionepose_amd/csrc -o tools/phase_probe tools/phase_probe.hip
$HIPCC --offload-arch=gfx950 -O3 -std=c++17 -w -Ionepose_amd/csrc -o tools/pnp_probe tools/pnp_probe.hip
