#!/bin/bash
# DMA (W planes by global_load_lds) vs register-staged bf16-mode GEMMs: tests of the bf16 modes,
# then config 2 in fp32 / fp32_split (DMA on and off) and config 5 bf16 (DMA on and off).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_matcher_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "split or bf16 or fixture or cache or tables or prec" > gpurun_out/dma_tests.log 2>&1 || { tail -30 gpurun_out/dma_tests.log; exit 1; }
tail -1 gpurun_out/dma_tests.log
run() {   # name, env, args
  env $2 timeout -k 10 200 python bench.py --steps 300 --warmup 5 --no-cpu-baseline $3 > gpurun_out/ab_$1.json 2> gpurun_out/ab_$1.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/ab_$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$1', d['value'], d['roofline']['avg_launch_us'], d['roofline']['alone']['avg_launch_us'], {x: k[x] for x in ('mlp1_gemm','qkv_gemm','mlp2_gemm','kv_reduce')})"
}
run fp32 ONEPOSE_GEMM_DMA=1 "--precision fp32"
run split_dma ONEPOSE_GEMM_DMA=1 "--precision fp32_split"
run split_reg ONEPOSE_GEMM_DMA=0 "--precision fp32_split"
run fp32b ONEPOSE_GEMM_DMA=1 "--precision fp32"
run split_dmab ONEPOSE_GEMM_DMA=1 "--precision fp32_split"
run c5_dma ONEPOSE_GEMM_DMA=1 "--precision bf16 --n1 2048 --n3 8192"
run c5_reg ONEPOSE_GEMM_DMA=0 "--precision bf16 --n1 2048 --n3 8192"
