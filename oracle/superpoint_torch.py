"""ORACLE -- test infrastructure only.  Never imported by the product path.

PyTorch-CPU restatement (float32) of SuperPoint's forward
(``src/models/extractors/SuperPoint/superpoint.py:170-243``): conv2d backbone, softmax score
head + pixel shuffle, ``simple_nms`` by max-pools (:47-64), threshold, ``remove_borders``
(:66-76), ``top_k_keypoints`` (:78-93) and bilinear ``sample_descriptors`` (:95-113,
``grid_sample`` with torch 2.x's default align_corners=False).  ``bench.py``'s e2e
``cpu_baseline`` times it with every host thread it is given.  Pinned by
``tests/test_superpoint_oracle.py`` against the reference's fixtures.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def to_torch(sd):
    return {k: torch.from_numpy(np.ascontiguousarray(v, np.float32)) for k, v in sd.items()}


def _cv(sd, name, x):
    w = sd[name + ".weight"]
    return F.conv2d(x, w, sd[name + ".bias"], padding=w.shape[-1] // 2)


def _nms(scores, r):
    def mp(x):
        return F.max_pool2d(x, kernel_size=2 * r + 1, stride=1, padding=r)
    zeros = torch.zeros_like(scores)
    max_mask = scores == mp(scores)
    for _ in range(2):
        supp = mp(max_mask.float()) > 0
        ss = torch.where(supp, zeros, scores)
        max_mask = max_mask | ((ss == mp(ss)) & ~supp)
    return torch.where(max_mask, scores, zeros)


@torch.no_grad()
def forward(sd, img, nms_radius=4, keypoint_threshold=0.005, remove_borders=4,
            max_keypoints=-1):
    """One image [H,W] -> (keypoints [n,2] (x, y), scores [n], descriptors [256,n]), plus the
    score map [H,W]."""
    x = torch.as_tensor(img, dtype=torch.float32)[None, None]
    relu = F.relu
    x = F.max_pool2d(relu(_cv(sd, "conv1b", relu(_cv(sd, "conv1a", x)))), 2, 2)
    x = F.max_pool2d(relu(_cv(sd, "conv2b", relu(_cv(sd, "conv2a", x)))), 2, 2)
    x = F.max_pool2d(relu(_cv(sd, "conv3b", relu(_cv(sd, "conv3a", x)))), 2, 2)
    x = relu(_cv(sd, "conv4b", relu(_cv(sd, "conv4a", x))))
    s = F.softmax(_cv(sd, "convPb", relu(_cv(sd, "convPa", x))), 1)[:, :-1]
    b, _, h, w = s.shape
    smap = s.permute(0, 2, 3, 1).reshape(b, h, w, 8, 8).permute(0, 1, 3, 2, 4).reshape(h * 8, w * 8)
    nms = _nms(smap[None, None], nms_radius)[0, 0]
    yx = torch.nonzero(nms > keypoint_threshold)
    sc = nms[yx[:, 0], yx[:, 1]]
    H, W = smap.shape
    bd = remove_borders
    ok = (yx[:, 0] >= bd) & (yx[:, 0] < H - bd) & (yx[:, 1] >= bd) & (yx[:, 1] < W - bd)
    yx, sc = yx[ok], sc[ok]
    if 0 <= max_keypoints < len(yx):
        sc, idx = torch.topk(sc, max_keypoints, dim=0)
        yx = yx[idx]
    kp = torch.flip(yx, [1]).float()
    d = F.normalize(_cv(sd, "convDb", relu(_cv(sd, "convDa", x))), p=2, dim=1)
    s8 = 8
    g = (kp - s8 / 2 + 0.5) / torch.tensor([w * s8 - s8 / 2 - 0.5, h * s8 - s8 / 2 - 0.5])
    g = (g * 2 - 1).view(1, 1, -1, 2)
    desc = F.normalize(F.grid_sample(d, g, mode="bilinear", align_corners=False).reshape(256, -1),
                       p=2, dim=0)
    return kp.numpy(), sc.numpy(), desc.numpy(), smap.numpy()
