"""SuperPoint timing on one GPU: the HIP detector (eager launches and a captured HIP graph)
against the same network run as plain PyTorch ops on the same device (MIOpen convs, the
reference's superpoint.py op sequence), at OnePose's 512x512 crop size.

    python tools/sp_bench.py [--batch 1 8] [--iters 50]
Prints one JSON line per batch size."""
import argparse
import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onepose_amd import synthetic  # noqa: E402
from onepose_amd.superpoint import SuperPoint  # noqa: E402


def torch_superpoint(sd, img, max_kp):
    """superpoint.py:170-243 as torch ops (the reference's GPU path, MIOpen convs)."""
    def cv(n, x, p=1):
        return F.conv2d(x, sd[f"{n}.weight"], sd[f"{n}.bias"], padding=p)
    r = torch.relu
    x = F.max_pool2d(r(cv("conv1b", r(cv("conv1a", img)))), 2)
    x = F.max_pool2d(r(cv("conv2b", r(cv("conv2a", x)))), 2)
    x = F.max_pool2d(r(cv("conv3b", r(cv("conv3a", x)))), 2)
    x = r(cv("conv4b", r(cv("conv4a", x))))
    s = F.softmax(cv("convPb", r(cv("convPa", x)), 0), 1)[:, :-1]
    b, _, h, w = s.shape
    s = s.permute(0, 2, 3, 1).reshape(b, h, w, 8, 8).permute(0, 1, 3, 2, 4).reshape(b, h * 8, w * 8)

    def mp(t):
        return F.max_pool2d(t, 7, 1, 3)
    z = torch.zeros_like(s)
    mm = s == mp(s)
    for _ in range(2):
        sp = mp(mm.float()) > 0
        ss = torch.where(sp, z, s)
        mm = mm | ((ss == mp(ss)) & ~sp)
    s = torch.where(mm, s, z)
    d = F.normalize(cv("convDb", r(cv("convDa", x)), 0), p=2, dim=1)
    out = []
    for i in range(b):
        k = torch.nonzero(s[i] > 0.005)
        sc = s[i][tuple(k.t())]
        m = (k[:, 0] >= 4) & (k[:, 0] < h * 8 - 4) & (k[:, 1] >= 4) & (k[:, 1] < w * 8 - 4)
        k, sc = k[m], sc[m]
        if max_kp < len(k):
            sc, idx = torch.topk(sc, max_kp, dim=0)
            k = k[idx]
        k = torch.flip(k, [1]).float()
        kk = k - 4 + 0.5
        kk = kk / torch.tensor([w * 8 - 4 - 0.5, h * 8 - 4 - 0.5], device=k.device)
        kk = kk * 2 - 1
        desc = F.grid_sample(d[i:i + 1], kk.view(1, 1, -1, 2), mode="bilinear",
                             align_corners=False)
        out.append(F.normalize(desc.reshape(1, 256, -1), p=2, dim=1))
    return out


def timed(fn, iters):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--size", type=int, default=512)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    sdn = synthetic.superpoint_state_dict(0)
    sdt = {k: torch.from_numpy(v).to(dev) for k, v in sdn.items()}
    m = SuperPoint({"nms_radius": 3, "max_keypoints": 4096}).to(dev)
    m.load_state_dict(sdn)
    for b in a.batch:
        imgs = np.stack([synthetic.superpoint_image(a.size, a.size, s) for s in range(b)])
        img = torch.from_numpy(imgs)[:, None].to(dev)
        eager = timed(lambda: m.detect_raw(img), a.iters)
        # graph: the raw launch sequence with fixed outputs
        raw = m.detect_raw(img)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m.detect_raw(img)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                raw = m.detect_raw(img)
        torch.cuda.current_stream().wait_stream(s)
        graph = timed(g.replay, a.iters)
        with torch.no_grad():
            ref = timed(lambda: torch_superpoint(sdt, img, 4096), max(5, a.iters // 5))
        print(json.dumps({"batch": b, "size": a.size, "hip_eager_ms": round(eager, 4),
                          "hip_graph_ms": round(graph, 4), "torch_ref_ms": round(ref, 4),
                          "images_per_s_graph": round(b * 1000 / graph, 1),
                          "keypoints": raw["counts"].tolist()}), flush=True)


if __name__ == "__main__":
    main()
