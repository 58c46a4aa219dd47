#!/bin/bash
# Round 4: config-5 oracle test, the bench's N>1 path rehearsed with 2 ranks on the one GPU
# (gloo, ONEPOSE_REHEARSE_ONE_GPU=1: sharding + gather + frame order, not a scaling number),
# then the default bench line.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04_b}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k config5 > $O/c5_test.log 2>&1 || { tail -30 $O/c5_test.log; exit 1; }
grep -E "config 5|passed|failed" $O/c5_test.log
ONEPOSE_REHEARSE_ONE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > $O/rehearse2.json 2> $O/rehearse2.err || { tail -30 $O/rehearse2.err; exit 1; }
tail -1 $O/rehearse2.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rehearse2', d['value'], d['n_gpus'], d['config']['global_batch'], d['pose'])"
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20.json 2> $O/bench_20.err || exit $?
tail -1 $O/bench_20.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench20', d['value'], d['ms_per_step'], d['roofline']['frac'], d['pose'], d.get('cpu_baseline'))"
