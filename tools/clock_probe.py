"""Dev probe (not shipped): ms/step of the serial pipeline in chunks of 10 steps right after a
3-step warmup, to see whether a freshly idle GPU needs sustained load before full speed."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onepose_amd import matcher, synthetic  # noqa: E402
from onepose_amd.pipeline import FramePipeline  # noqa: E402

dev = torch.device("cuda", 0)
sd = synthetic.make_state_dict(0)
data, obj, frames = synthetic.make_matcher_inputs(1024, 4096, 8, seed=0)
pipe = FramePipeline(matcher.from_state_dict(sd), data["keypoints3d"][0],
                     data["descriptors3d_db"][0], data["descriptors2d_db"][0], 1, 1024, dev)
pipe.set_frames(data["descriptors2d_query"], data["keypoints2d"],
                np.stack([f.K for f in frames]), np.stack([f.pose_gt for f in frames]))
g = pipe.capture(0)
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
t_start = time.perf_counter()
out = []
for c in range(int(sys.argv[1]) if len(sys.argv) > 1 else 40):  # noqa
    t0 = time.perf_counter()
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    out.append(f"{(time.perf_counter() - t_start) * 1e3:.0f}ms:{(time.perf_counter() - t0) * 100:.3f}")
    if c == 19 and len(sys.argv) <= 2:
        time.sleep(2.0)   # idle gap: does the GPU drop back?
        out.append("sleep2s")
print(" ".join(out))
