#!/bin/bash
# Round 6: the N > 1 bench path (RCCL process group, barrier, all-gather) at world size 1 on one
# GPU (ONEPOSE_FORCE_PG=1 under torch.distributed.run) against the plain one-process line.
set -o pipefail
O=gpurun_out/r06pg1
mkdir -p $O
pg() {   # name, args
  ONEPOSE_FORCE_PG=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --no-cpu-baseline $2 \
    > $O/$1.json 2> $O/$1.err || exit 1
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'])"
}
one() {
  timeout -k 10 200 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || exit 1
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'])"
}
for i in 1 2; do
  pg pg_s300_$i "--steps 300"
  one plain_s300_$i "--steps 300"
  pg pg_s20_$i "--steps 20 --warmup 5"
  one plain_s20_$i "--steps 20 --warmup 5"
done
pg pg_base_s300 "--steps 300 --no-staged-inputs"
