set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for args in "--batch 1 --match-streams 1" "--batch 1 --match-streams 2" "--batch 2 --match-streams 1" "--batch 2 --match-streams 2" "--batch 1 --match-streams 2 --precision fp32_split"; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-cpu-baseline $args > gpurun_out/bb.json 2> gpurun_out/bb.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/bb.json').read().strip().splitlines()[-1]); print('$args', d['value'], d['roofline']['avg_launch_us'], d['kernel_ms_per_step'])"
done
