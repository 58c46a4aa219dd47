#!/bin/bash
# N > 1 code path on a one-GPU box (every rank on device 0 over gloo; not a scaling number):
# torchrun at 2 and 4 ranks, the driver's 20-step command.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-rehearse}
mkdir -p $O
for n in 2 4; do
  ONEPOSE_REHEARSE_ONE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n \
    --steps 20 --warmup 5 > $O/rehearse_$n.json 2> $O/rehearse_$n.err || { tail -20 $O/rehearse_$n.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/rehearse_$n.json').read().strip().splitlines()[-1]); print($n, d['value'], d['n_gpus'], d['config'], d.get('rehearsal'))"
done
