"""Dev tool: where a drop-in GATsSuperGlue.forward call's time goes (config 2, B = 1), object
resident or not: the whole call, packed_weights, _resident, and the library call alone."""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from onepose_amd import matcher, synthetic


def clock(fn, n=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


dev = torch.device("cuda", 0)
m = matcher.from_state_dict(synthetic.make_state_dict(0)).to(dev)
data, _, _ = synthetic.make_matcher_inputs(1024, 4096, 8, seed=3)
t = {k: torch.from_numpy(v).to(dev) for k, v in data.items()}
with torch.no_grad():
    for res in (True, False):
        m.resident_object = res
        print(f"resident={res}: forward {clock(lambda: m(t)):.3f} ms")
    m.resident_object = True
    print(f"packed_weights {clock(lambda: m.packed_weights(dev)):.3f} ms")
    print(f"_weight_tensors {clock(lambda: m._weight_tensors()):.3f} ms")
    # ragged n1 (the entry bench's frames: 1024 - (37 i mod 97)), the object fixed
    ts = []
    for i in range(12):
        n1 = 1024 - (37 * i) % 97
        d = dict(t)
        d["descriptors2d_query"] = t["descriptors2d_query"][:, :, :n1].contiguous()
        d["keypoints2d"] = t["keypoints2d"][:, :n1].contiguous()
        ts.append(d)
    for rep in range(2):
        torch.cuda.synchronize()
        s0 = time.perf_counter()
        for d in ts:
            m(d)
        torch.cuda.synchronize()
        print(f"ragged n1, pass {rep}: {(time.perf_counter() - s0) / len(ts) * 1e3:.3f} ms per forward")
    import cProfile, pstats
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(10):
        m(t)
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(18)
