set -u
bash tools/gpu_configs.sh && bash tools/gpu_pmc.sh && bash tools/gpu_sq.sh && STEPS=20 bash tools/gpu_prof.sh
