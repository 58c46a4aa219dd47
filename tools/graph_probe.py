"""Dev probe (not shipped): per-step time of the config-2 pipeline under eager launches,
one graph replayed K times, and K distinct graphs (cold / after one warm replay each)."""
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
m = matcher.from_state_dict(sd)
pipe = FramePipeline(m, data["keypoints3d"][0], data["descriptors3d_db"][0],
                     data["descriptors2d_db"][0], 1, 1024, dev, scale=1000.0)
pipe.set_frames(data["descriptors2d_query"], data["keypoints2d"],
                np.stack([f.K for f in frames]), np.stack([f.pose_gt for f in frames]))
K = 30


def timed(fn, label):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    th = (time.perf_counter() - t0) / K * 1e3
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K * 1e3
    print(f"{label:40s} {dt:.4f} ms/step  (host enqueue {th:.4f})", flush=True)


def eager():
    for _ in range(K):
        pipe.enqueue()


for _ in range(5):
    pipe.enqueue()
timed(eager, "eager")
timed(eager, "eager again")
g = pipe.capture(0)
g.replay()
timed(lambda: [g.replay() for _ in range(K)], "one graph x K")
pool = torch.cuda.graph_pool_handle()
gs = [pipe.capture(0, pool) for _ in range(K)]
timed(lambda: [x.replay() for x in gs], "K graphs, cold")
timed(lambda: [x.replay() for x in gs], "K graphs, warm")
timed(eager, "eager again")
timed(lambda: [g.replay() for _ in range(K)], "one graph x K again")
