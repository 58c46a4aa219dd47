#!/bin/bash
# Pose-stream priority A/B at config 2 (fp32): default vs high priority, 300 and 20 steps.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-prio}
mkdir -p $O
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
run() {   # name, args
  timeout -k 10 200 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$1', d['value'], {x: k[x] for x in ('mlp1_gemm','pnp_ransac','pnp_refit')})"
}
for i in 1 2; do
  run p0_$i "--steps 300 --warmup 5"
  run ph_$i "--steps 300 --warmup 5 --pose-priority -1"
done
for i in 1 2; do
  run s20_p0_$i "--steps 20 --warmup 5"
  run s20_ph_$i "--steps 20 --warmup 5 --pose-priority -1"
done
