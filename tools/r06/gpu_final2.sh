#!/bin/bash
# Round 6, second measurement set (the staged schedule): the full gpu_final.sh set into
# gpurun_out/r06final2 (GPU suite, default line + CPU baseline, 20-step lines, other configs,
# rocprof, PMC, SQ, N=2 rehearsal, entry path, pose probe).
OUT=${OUT:-r06final2} exec ./tools/r06/gpu_final.sh
