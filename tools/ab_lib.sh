set -u
for r in 1 2 3; do for v in base q64; do if [ $v = base ]; then lib=""; else lib=$PWD/tools/ab/lib_$v.so; fi
ONEPOSE_LIB=$lib timeout -k 10 200 python bench.py --steps 500 --warmup 20 --no-cpu-baseline > gpurun_out/ab.json 2>/dev/null || exit 1
python -c "import json;d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]);k=d['kernel_ms_per_step'];print('$v',d['value'],k['qkv_gemm'],k['kv_reduce'])"; done; done
