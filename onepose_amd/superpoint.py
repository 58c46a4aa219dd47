"""SuperPoint descriptor sampling on libonepose_hip.

``sample_descriptors(keypoints, descriptors, s=8)`` is the drop-in for
``src/models/extractors/SuperPoint/superpoint.py:95-113``: bilinear interpolation of the
dense descriptor map at the keypoints (zero padding), then L2 normalisation over channels.
``align_corners`` defaults to the reference's own rule -- ``int(torch.__version__[2]) > 2``
(superpoint.py:108), i.e. True on the pinned torch 1.8 and False on torch 2.x -- and can be
forced either way.  The SuperPoint backbone itself is out of this round's scope (SURVEY.md
§8f rank 1).
"""
from __future__ import annotations

import torch

from . import _lib


def reference_align_corners() -> bool:
    return int(torch.__version__[2]) > 2


def sample_descriptors(keypoints, descriptors, s: int = 8, align_corners=None):
    """keypoints [b, n, 2] (x, y) pixels, descriptors [b, c, h, w] -> [b, c, n]."""
    if align_corners is None:
        align_corners = reference_align_corners()
    if descriptors.device.type != "cuda":
        raise RuntimeError("onepose_amd.sample_descriptors runs on a ROCm GPU only")
    lib = _lib.load()
    b, c, h, w = descriptors.shape
    n = keypoints.shape[1]
    kp = keypoints.float().contiguous()
    d = descriptors.float().contiguous()
    out = torch.empty(b, c, n, dtype=torch.float32, device=d.device)
    _lib.check(lib.onepose_sample_descriptors(kp.data_ptr(), d.data_ptr(), b, n, c, h, w, int(s),
                                              int(bool(align_corners)), out.data_ptr(),
                                              _lib.stream_ptr(d.device)), "sample_descriptors")
    return out
