#!/bin/bash
# What the pose stage costs the matcher streams: config 2 with and without it (diagnostic),
# alternating, 300 and 20 steps.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-nopose}
mkdir -p $O
run() {   # name, args
  timeout -k 10 200 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$1', d['value'], k['mlp1_gemm'])"
}
for i in 1 2; do
  run pose_$i "--steps 300 --warmup 5"
  run nopose_$i "--steps 300 --warmup 5 --diag-no-pose"
done
for i in 1 2 3; do
  run s20_pose_$i "--steps 20 --warmup 5"
  run s20_nopose_$i "--steps 20 --warmup 5 --diag-no-pose"
done
