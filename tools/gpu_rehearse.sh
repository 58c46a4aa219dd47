#!/bin/bash
# 2-rank rehearsal of the multi-GPU bench path with both ranks on the one GPU (gloo), twice,
# with the current library and with tools/ab/lib_prev.so.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in cur prev; do
  if [ $v = cur ]; then lib=""; else lib=$PWD/tools/ab/lib_prev.so; fi
  ONEPOSE_LIB=$lib ONEPOSE_REHEARSE_ONE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 50 --warmup 5 --no-cpu-baseline \
    > gpurun_out/reh_$v.json 2> gpurun_out/reh_$v.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/reh_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d.get('diag'))"
done
