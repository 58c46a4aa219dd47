#!/bin/bash
# The driver's multi-GPU launcher path at N = 1 on the one-GPU box: torch.distributed.run with
# one rank (RCCL init, the timed region's barrier / max-over-ranks, the result gather).
set -u
export TMPDIR=/tmp
O=gpurun_out/r04v
mkdir -p $O
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 > $O/torchrun_n1.json 2> $O/torchrun_n1.err || { tail -20 $O/torchrun_n1.err; exit 1; }
python -c "import json; d=json.loads(open('$O/torchrun_n1.json').read().strip().splitlines()[-1]); print('torchrun N=1', d['value'], d['n_gpus'], d['config']['parallelism'], d['pose'])"
