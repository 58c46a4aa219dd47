#!/bin/bash
# Round-6 measurement set on the committed build: GPU suite, the default bench line (with the
# CPU baseline), the driver's 20-step line twice, the other precisions / configs, a rocprofv3
# kernel-trace/stats pass, PMC HBM traffic (FETCH_SIZE / WRITE_SIZE in separate passes) and the
# SQ counters for config 2.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06final}
mkdir -p $O
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
fi
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
python -c "import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); print('default', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'))"
for i in 1 2; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_20_$i.json 2> $O/bench_20_$i.err || exit $?
python -c "import json; d=json.loads(open('$O/bench_20_$i.json').read().strip().splitlines()[-1]); print('20 steps', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
run() {   # name, args
  timeout -k 10 300 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
}
run c2_split "--precision fp32_split --steps 300 --warmup 5"
run c2_bf16 "--precision bf16 --steps 300 --warmup 5"
run c5_bf16 "--n1 2048 --n3 8192 --precision bf16 --desc-dtype fp16 --steps 100 --warmup 3"
run c5_bf16_f32desc "--n1 2048 --n3 8192 --precision bf16 --steps 100 --warmup 3"
run c3 "--n3 16384 --batch 32 --steps 10 --warmup 2"
run c4 "--n3 2500 --batch 32 --steps 10 --warmup 2"
mkdir -p $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline > $O/prof/bench.json 2> $O/prof/bench.err || exit $?
echo prof ok
mkdir -p $O/pmc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc/$c -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --serial --eager \
    > $O/pmc/bench_$c.json 2> $O/pmc/bench_$c.err || exit $?
  echo "pmc $c ok"
done
python3 tools/pmc_summary.py $O/pmc > $O/pmc/pmc_traffic.json || exit $?
mkdir -p $O/sq
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $O/sq/raw -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --serial --eager \
  > $O/sq/bench.json 2> $O/sq/bench.err || exit $?
python3 tools/pmc_summary.py --sq $O/sq/raw > $O/sq/sq_summary.json || exit $?
echo "sq ok"
# config 5's counters (fp16 descriptors): transpose_in reads half the bytes
mkdir -p $O/pmc_c5
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_c5/$c -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --serial --eager --n1 2048 --n3 8192 \
    --precision bf16 --desc-dtype fp16 > $O/pmc_c5/bench_$c.json 2> $O/pmc_c5/bench_$c.err || exit $?
done
python3 tools/pmc_summary.py $O/pmc_c5 > $O/pmc_c5/pmc_traffic.json || exit $?
mkdir -p $O/sq_c5
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $O/sq_c5/raw -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --serial --eager --n1 2048 --n3 8192 \
  --precision bf16 --desc-dtype fp16 > $O/sq_c5/bench.json 2> $O/sq_c5/bench.err || exit $?
python3 tools/pmc_summary.py --sq $O/sq_c5/raw > $O/sq_c5/sq_summary.json || exit $?
echo "c5 counters ok"
# the N > 1 code path (sharding, gather, global frame order) on real HIP results: 2 ranks, gloo
# (two processes on one GPU: eight hardware queues each, or their streams share queues --
# profiles/r06/hwq/; the driver's multi-GPU run is one process per GPU)
GPU_MAX_HW_QUEUES=8 ONEPOSE_REHEARSE_ONE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 \
  --warmup 5 --no-cpu-baseline > $O/rehearse_n2.json 2> $O/rehearse_n2.err || exit $?
tail -1 $O/rehearse_n2.json
timeout -k 10 600 python -u tools/entry_bench.py --frames 64 --n3 4096 --out $O/entry.json > $O/entry.log 2>&1 || { tail -30 $O/entry.log; exit 1; }
grep -E "^(superpoint|detections)" $O/entry.log
# the pose stage's phases on the final build
timeout -k 10 60 ./tools/pnp_probe 900 0.1 > $O/pnp_probe_900.txt 2>&1 || exit 1
timeout -k 10 60 ./tools/pnp_probe 300 0.0 > $O/pnp_probe_300.txt 2>&1 || exit 1
grep event $O/pnp_probe_*.txt
