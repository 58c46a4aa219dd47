#!/bin/bash
# Pose-stage iteration: phases (tools/pnp_probe), then the pose tests against the C oracle.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06pose}
mkdir -p $O
timeout -k 10 60 ./tools/pnp_probe 900 0.1 > $O/pnp_probe_900.txt 2>&1 || { cat $O/pnp_probe_900.txt; exit 1; }
timeout -k 10 60 ./tools/pnp_probe 300 0.0 > $O/pnp_probe_300.txt 2>&1 || { cat $O/pnp_probe_300.txt; exit 1; }
cat $O/pnp_probe_900.txt $O/pnp_probe_300.txt
timeout -k 10 600 python -u -m pytest tests/test_pnp_gpu.py tests/test_frame_ops_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 300 --timeout-method thread ${PYARGS:-} > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
