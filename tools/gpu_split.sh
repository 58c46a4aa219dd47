set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_matcher_gpu.py -x -q -s --timeout 200 > gpurun_out/t.log 2>&1; rc=$?
tail -3 gpurun_out/t.log; grep "max |conf" gpurun_out/t.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for prec in fp32 fp32_split fp32 fp32_split; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --precision $prec > gpurun_out/p_$prec.json 2> gpurun_out/p_$prec.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/p_$prec.json').read().strip().splitlines()[-1]); print('$prec', d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_us'], list(d['kernel_ms_per_step'].items())[:5], d['pose']['cmd5'])"
done
