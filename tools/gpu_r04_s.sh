#!/bin/bash
# The config-5 counter passes (gpu_r04_r.sh), then the two-stream kernel trace of the final
# build (gpu_r04_timeline.sh into gpurun_out/r04tl).
set -u
bash tools/gpu_r04_r.sh || exit $?
OUT=r04tl bash tools/gpu_r04_timeline.sh
