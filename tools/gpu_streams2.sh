set -u
export TMPDIR=/tmp
for r in 1 2; do
for ms in 2 3 4; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-cpu-baseline --match-streams $ms > gpurun_out/ms$ms.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/ms$ms.json').read().strip().splitlines()[-1]); print('streams $ms', d['value'])"
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-cpu-baseline --match-streams $ms > gpurun_out/ms$ms.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/ms$ms.json').read().strip().splitlines()[-1]); print('streams $ms q8', d['value'])"
done
done
