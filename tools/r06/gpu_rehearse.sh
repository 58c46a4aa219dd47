#!/bin/bash
# Round 6: the 2-rank one-GPU rehearsal of the N > 1 bench under the staged schedule -- staged vs
# unstaged, and staged with more hardware queues per process (GPU_MAX_HW_QUEUES=8).
set -o pipefail
O=gpurun_out/r06reh
mkdir -p $O
reh() {   # name, env, args
  env ONEPOSE_REHEARSE_ONE_GPU=1 $2 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 \
    --warmup 5 --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || exit 1
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'])"
}
reh staged "" ""
reh base "" "--no-staged-inputs"
reh staged_q8 "GPU_MAX_HW_QUEUES=8" ""
reh s15 "" "--staged-split 15"
