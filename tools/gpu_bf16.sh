#!/bin/bash
# bf16-attention mode: parity-vs-fp32 tests, then fp32 / bf16 benches (config 2) and config 5.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_matcher_gpu.py -q -rf -x --timeout=300 -k "bf16 or prepared" > gpurun_out/bf16_tests.log 2>&1
rc=$?
tail -8 gpurun_out/bf16_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for p in fp32 bf16; do
  timeout -k 10 300 python bench.py --precision $p --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$p.json 2> gpurun_out/bench_$p.err || exit $?
done
timeout -k 10 300 python bench.py --precision bf16 --n1 2048 --n3 8192 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c5_bf16.json 2> gpurun_out/bench_c5_bf16.err || exit $?
timeout -k 10 300 python bench.py --precision fp32 --n1 2048 --n3 8192 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c5_fp32.json 2> gpurun_out/bench_c5_fp32.err || exit $?
python - <<'PY'
import json
for f in ("bench_fp32", "bench_bf16", "bench_c5_fp32", "bench_c5_bf16"):
    d = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f, d["value"], d["ms_per_step"], r["kernel"], r["avg_launch_us"], r["frac"], d["pose"]["cmd5"])
    print("   ", {k: v for k, v in list(d["kernel_ms_per_step"].items())[:8]})
PY
