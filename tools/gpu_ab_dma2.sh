#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 150 ./tools/split_probe > gpurun_out/split_probe3.txt 2>&1 || exit $?
grep -A9 "production kernels" gpurun_out/split_probe3.txt
timeout -k 10 300 python -u -m pytest tests/test_matcher_gpu.py tests/test_sharded_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "split or bf16 or fixture or cache or tables or prec or sharded" > gpurun_out/dma2_tests.log 2>&1 || { tail -30 gpurun_out/dma2_tests.log; exit 1; }
tail -1 gpurun_out/dma2_tests.log
run() {
  timeout -k 10 200 python bench.py --steps 300 --warmup 5 --no-cpu-baseline $2 > gpurun_out/ab_$1.json 2> gpurun_out/ab_$1.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/ab_$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$1', d['value'], d['roofline']['avg_launch_us'], d['roofline']['alone']['avg_launch_us'], {x: k[x] for x in ('mlp1_gemm','qkv_gemm','mlp2_gemm','kv_reduce')})"
}
run fp32 "--precision fp32"
run split "--precision fp32_split"
run fp32b "--precision fp32"
run splitb "--precision fp32_split"
run c5 "--precision bf16 --n1 2048 --n3 8192"
