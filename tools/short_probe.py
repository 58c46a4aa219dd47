"""Why does the first 20-step timed region read slower than repeats?  Times 20-step regions
of the bench's default schedule under different preludes (GPU idle, stamp re-arm, ...)."""
import os, sys, time, json
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from onepose_amd import _lib, matcher, synthetic
from onepose_amd.pipeline import FramePipeline

dev = torch.device("cuda", 0)
lib = _lib.load()
B, n1, n3, L = 1, 1024, 4096, 8
sd = synthetic.make_state_dict(0)
data, obj, frames = synthetic.make_matcher_inputs(n1, n3, L, seed=0, batch=B)
m = matcher.from_state_dict(sd, {**synthetic.DEFAULT_HPARAMS, "attention_precision": "fp32"})
pipe = FramePipeline(m, data["keypoints3d"][0], data["descriptors3d_db"][0],
                     data["descriptors2d_db"][0], B, n1, dev, scale=1000.0, slots=3)
pipe.set_frames(data["descriptors2d_query"], data["keypoints2d"],
                np.stack([f.K for f in frames]), np.stack([f.pose_gt for f in frames]))
for _ in range(5):
    pipe.enqueue()
torch.cuda.synchronize()
g = pipe.capture_stages(torch.cuda.graph_pool_handle())
pipe.run_stream(3, graphs=g, match_streams=2)
torch.cuda.synchronize()
K = int(os.environ.get("K", "20"))

def region(tag, prelude=None):
    if prelude:
        prelude()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pipe.run_stream(K, graphs=g, match_streams=2)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K * 1e3
    print(f"{tag:28s} {dt:.4f} ms/step", flush=True)
    return dt

def idle(ms):
    return lambda: (torch.cuda.synchronize(), time.sleep(ms / 1e3))

def busy_prelude():
    pipe.run_stream(6, graphs=g, match_streams=2)

for rep in range(2):
    region("back-to-back")
    region("back-to-back")
    region("idle 1 ms", idle(1))
    region("idle 5 ms", idle(5))
    region("idle 20 ms", idle(20))
    region("idle 100 ms", idle(100))
    region("idle 500 ms", idle(500))
    region("after 6-step prelude", busy_prelude)
