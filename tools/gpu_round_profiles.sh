#!/bin/bash
# Round-end measurement set (one box): default bench line, the harness's 20-step line, a
# rocprofv3 kernel-trace/stats pass, PMC HBM traffic (separate passes), and a 2-rank rehearsal
# of the multi-GPU path on the one device (gloo).  Everything lands in gpurun_out/round/.
set -u
export TMPDIR=/tmp
O=gpurun_out/round
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
tail -1 $O/bench_default.json | cut -c1-200
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_20.json 2> $O/bench_20.err || exit $?
tail -1 $O/bench_20.json | cut -c1-200
mkdir -p $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline > $O/prof/bench.json 2> $O/prof/bench.err || exit $?
echo prof ok
mkdir -p $O/pmc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc/$c -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --serial --eager \
    > $O/pmc/bench_$c.json 2> $O/pmc/bench_$c.err || exit $?
  echo "pmc $c ok"
done
python3 tools/pmc_summary.py $O/pmc > $O/pmc/traffic.json || exit $?
ONEPOSE_REHEARSE_ONE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 50 --warmup 5 --no-cpu-baseline \
  > $O/bench_rehearse2.json 2> $O/bench_rehearse2.err || exit $?
tail -1 $O/bench_rehearse2.json | cut -c1-200
