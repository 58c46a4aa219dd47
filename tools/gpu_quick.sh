set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/b.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['avg_launch_us'], d['kernel_ms_per_step'])"
