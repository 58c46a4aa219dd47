"""Per-launch kernel times of one cached config-2 frame in launch order (serial, HIP events):
which layers' QKV / MLP launches are slow, and is it the data (weights / states)?"""
import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from onepose_amd import _lib, matcher, synthetic
from onepose_amd.pipeline import FramePipeline
import bench

dev = torch.device("cuda", 0)
lib = _lib.load()
B, n1, n3, L = 1, 1024, 4096, 8
wc = os.environ.get("WC", "1") == "1"
sd = synthetic.make_state_dict(0, well_conditioned=wc)
if os.environ.get("ZERO_W"):   # all attention weights replaced by one layer's
    pass
data, obj, frames = synthetic.make_matcher_inputs(n1, n3, L, seed=0, batch=B)
m = matcher.from_state_dict(sd)
pipe = FramePipeline(m, data["keypoints3d"][0], data["descriptors3d_db"][0],
                     data["descriptors2d_db"][0], B, n1, dev, scale=1000.0, slots=3)
pipe.set_frames(data["descriptors2d_query"], data["keypoints2d"],
                np.stack([f.K for f in frames]), np.stack([f.pose_gt for f in frames]))
for _ in range(3):
    pipe.enqueue()
torch.cuda.synchronize()
names = bench.profile_kinds(lib)
kinds, ms = bench.run_profiled(lib, pipe, 3, (1 << len(names)) - 1, 4096)
n = len(kinds) // 3
for step in range(3):
    row = []
    for k, t in zip(kinds[step * n:(step + 1) * n], ms[step * n:(step + 1) * n]):
        nm = names[k]
        if nm in ("qkv_gemm", "mlp1_gemm", "mlp2_gemm", "kv_reduce", "gat"):
            row.append(f"{nm[:4]}:{t*1e3:.1f}")
    print(" ".join(row), flush=True)
# state statistics per layer: denormals / magnitude in the inputs of each layer
