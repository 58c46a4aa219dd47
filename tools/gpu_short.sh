set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --diag-repeats 6 > gpurun_out/s20_$i.json 2> gpurun_out/s20_$i.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/s20_$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('diag_ms_per_step'))"
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --stage-marks > gpurun_out/s20_m.json 2> gpurun_out/s20_m.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/s20_m.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('stage_ms'))"
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --diag-steps > gpurun_out/s20_d.json 2> gpurun_out/s20_d.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/s20_d.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('diag_ms_per_step'))"
