"""ORACLE -- test infrastructure only.  Never imported by the product path.

CPU restatement (numpy) of SuperPoint's forward
(``src/models/extractors/SuperPoint/superpoint.py:170-243``) and its helpers ``simple_nms``
(:47-64), ``remove_borders`` (:66-76), ``top_k_keypoints`` (:78-93) and
``sample_descriptors`` (:95-113, via ``matcher_np.sample_descriptors``).

Convolutions are im2col GEMMs accumulated in float64 and rounded to float32 per layer (the
reference's own fp32 conv sums in an unspecified order; float64 is the tightest CPU
statement of the same math).  NMS and selection are exact float32 comparisons, so given the
same score map they reproduce the reference bit for bit.  ``top_k`` breaks equal scores by
raster index (torch.topk leaves that order unspecified).

Pinning: ``tests/test_superpoint_oracle.py`` checks every stage against
``tests/golden/superpoint.npz``, produced by running the reference module itself with
seeded weights in the build container (``tests/golden/make_golden.py superpoint_case``).
"""
from __future__ import annotations

import numpy as np

from .matcher_np import sample_descriptors

F32 = np.float32
LAYERS = ("conv1a", "conv1b", "conv2a", "conv2b", "conv3a", "conv3b", "conv4a", "conv4b",
          "convPa", "convPb", "convDa", "convDb")


def conv2d(x, w, b):
    """nn.Conv2d(stride 1, padding k//2) on x [C,H,W]; w [O,C,k,k] -> [O,H,W] float32."""
    c, h, wd = x.shape
    o, _, k, _ = w.shape
    p = k // 2
    xp = np.pad(x.astype(np.float64), ((0, 0), (p, p), (p, p)))
    cols = np.empty((c, k, k, h, wd), np.float64)
    for dy in range(k):
        for dx in range(k):
            cols[:, dy, dx] = xp[:, dy:dy + h, dx:dx + wd]
    y = w.reshape(o, -1).astype(np.float64) @ cols.reshape(c * k * k, h * wd)
    return (y + b.astype(np.float64)[:, None]).astype(F32).reshape(o, h, wd)


def _relu(x):
    return np.maximum(x, F32(0))


def _pool(x):
    """MaxPool2d(2, 2) on [C,H,W]."""
    c, h, w = x.shape
    return x[:, :h // 2 * 2, :w // 2 * 2].reshape(c, h // 2, 2, w // 2, 2).max(axis=(2, 4))


def encoder(sd, img):
    """superpoint.py:173-185: img [H,W] -> x [128,H/8,W/8]."""
    def cv(name, x):
        return conv2d(x, sd[f"{name}.weight"], sd[f"{name}.bias"])
    x = img[None].astype(F32)
    x = _pool(_relu(cv("conv1b", _relu(cv("conv1a", x)))))
    x = _pool(_relu(cv("conv2b", _relu(cv("conv2a", x)))))
    x = _pool(_relu(cv("conv3b", _relu(cv("conv3a", x)))))
    return _relu(cv("conv4b", _relu(cv("conv4a", x))))


def score_map(sd, x):
    """superpoint.py:188-194: softmax over 65, drop the dustbin, pixel shuffle -> [8h, 8w]."""
    s = conv2d(_relu(conv2d(x, sd["convPa.weight"], sd["convPa.bias"])), sd["convPb.weight"],
               sd["convPb.bias"]).astype(np.float64)
    e = np.exp(s - s.max(axis=0, keepdims=True))
    p = (e / e.sum(axis=0, keepdims=True)).astype(F32)[:-1]       # [64, h, w]
    _, h, w = p.shape
    return p.reshape(8, 8, h, w).transpose(2, 0, 3, 1).reshape(h * 8, w * 8)


def dense_descriptors(sd, x):
    """superpoint.py:225-228: convDa, ReLU, convDb, L2-normalise over channels."""
    d = conv2d(_relu(conv2d(x, sd["convDa.weight"], sd["convDa.bias"])), sd["convDb.weight"],
               sd["convDb.bias"])
    n = np.sqrt((d.astype(np.float64) ** 2).sum(axis=0, keepdims=True))
    return (d / np.maximum(n, 1e-12)).astype(F32)


def _max_pool(x, r):
    """max_pool2d(kernel 2r+1, stride 1, padding r) with -inf padding, on [H,W]."""
    h, w = x.shape
    xp = np.full((h + 2 * r, w + 2 * r), -np.inf, dtype=x.dtype)
    xp[r:r + h, r:r + w] = x
    rows = np.lib.stride_tricks.sliding_window_view(xp, 2 * r + 1, axis=1).max(axis=-1)
    return np.lib.stride_tricks.sliding_window_view(rows, 2 * r + 1, axis=0).max(axis=-1)


def simple_nms(scores, r):
    """superpoint.py:47-64 on one score map [H,W] (float32, exact comparisons)."""
    zeros = np.zeros_like(scores)
    max_mask = scores == _max_pool(scores, r)
    for _ in range(2):
        supp = _max_pool(max_mask.astype(F32), r) > 0
        ss = np.where(supp, zeros, scores)
        new_max = ss == _max_pool(ss, r)
        max_mask = max_mask | (new_max & ~supp)
    return np.where(max_mask, scores, zeros)


def select_keypoints(nms, threshold, border, max_keypoints):
    """superpoint.py:197-212: threshold (raster order, torch.nonzero), remove_borders,
    top_k (descending; equal scores by raster index), flip to (x, y).
    Returns keypoints [n,2] float32 (x, y), scores [n]."""
    h, w = nms.shape
    yx = np.argwhere(nms > F32(threshold))
    sc = nms[yx[:, 0], yx[:, 1]]
    ok = ((yx[:, 0] >= border) & (yx[:, 0] < h - border) & (yx[:, 1] >= border)
          & (yx[:, 1] < w - border))
    yx, sc = yx[ok], sc[ok]
    if 0 <= max_keypoints < len(yx):
        order = np.lexsort((np.arange(len(sc)), -sc.astype(np.float64)))[:max_keypoints]
        yx, sc = yx[order], sc[order]
    return yx[:, ::-1].astype(F32), sc.astype(F32)


def forward(sd, img, nms_radius=4, keypoint_threshold=0.005, remove_borders=4,
            max_keypoints=-1, align_corners=False, record=None):
    """SuperPoint.forward for one image [H,W] -> (keypoints [n,2], scores [n], desc [256,n])."""
    x = encoder(sd, img)
    smap = score_map(sd, x)
    dense = dense_descriptors(sd, x)
    kp, sc = select_keypoints(simple_nms(smap, nms_radius), keypoint_threshold, remove_borders,
                              max_keypoints)
    desc = sample_descriptors(kp[None], dense[None], 8, align_corners)[0]
    if record is not None:
        record.update(score_map=smap, dense=dense)
    return kp, sc, desc
