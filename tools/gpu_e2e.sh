#!/bin/bash
# Pipeline tests (incl. the detector stage), then the default bench and the --e2e bench.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_pipeline_gpu.py tests/test_superpoint_gpu.py -q -rf -x --timeout=300 > gpurun_out/e2e_tests.log 2>&1
rc=$?
tail -8 gpurun_out/e2e_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps ${STEPS:-50} --warmup 5 --no-cpu-baseline > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
timeout -k 10 400 python bench.py --e2e --steps ${STEPS:-50} --warmup 5 ${E2E_ARGS:-} > gpurun_out/bench_e2e.json 2> gpurun_out/bench_e2e.err || exit $?
python - <<'PY'
import json
for f in ("gpurun_out/bench_default.json", "gpurun_out/bench_e2e.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d.get("detector"), d.get("cpu_baseline", {}).get("value"))
PY
