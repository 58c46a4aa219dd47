"""Round 6: the sequential value of matching_scores0[2] in test_resident_object_forward's data
(fp32_split), to tell which side of the rare side-stream mismatch deviates."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from onepose_amd import matcher, synthetic  # noqa: E402

dev = torch.device("cuda", 0)
sd = synthetic.make_state_dict(3)
hp = {**synthetic.DEFAULT_HPARAMS, "attention_precision": "fp32_split"}
res = matcher.from_state_dict(sd, hp).to(dev)
unc = matcher.from_state_dict(sd, hp).to(dev)
unc.resident_object = False
data, _, _ = synthetic.make_matcher_inputs(300, 1000, 8, seed=9)
t = {k: torch.from_numpy(v).to(dev) for k, v in data.items()}
g = torch.Generator().manual_seed(4)
for f in range(1, 3):   # the test's frame sequence, then its object edits
    t["descriptors2d_query"] = torch.nn.functional.normalize(
        torch.randn(t["descriptors2d_query"].shape, generator=g), dim=1).to(dev)
t["descriptors3d_db"].mul_(1.5)
t["descriptors2d_db"] = t["descriptors2d_db"].clone()
with torch.no_grad():
    for name, m in (("cached", res), ("uncached", unc)):
        p, c = m(t)
        torch.cuda.synchronize()
        v = p["matching_scores0"].cpu().numpy()
        print(name, " ".join("%.7e" % x for x in v[:8]), flush=True)
