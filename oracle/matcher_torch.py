"""ORACLE -- test infrastructure only.  Never imported by the product path.

PyTorch-CPU restatement (float32) of the GATsSPG matcher ``GATsSuperGlue.forward``
(``src/models/GATsSPG_architectures/GATs_SuperGlue.py:203-278``), op for op as the reference
runs it on the CPU: 1x1 ``conv1d`` projections (:112-120, :241-246), the einsum linear
attention (:88-99), ``cat`` + ``InstanceNorm1d`` + ``ReLU`` MLP (:135-147), the GAT layer with
its full ``h @ W`` GEMM and ``cat`` of the leaves (``GATs.py:62-123``), dual softmax and the
mutual nearest neighbour (:249-274).  ``bench.py``'s ``cpu_baseline`` times it with every
host thread it is given: the north star's "reference PyTorch-CPU path on the same box's host
cores" (the reference itself cannot travel to the GPU box).

Pinning: ``tests/test_oracle_golden.py`` checks it against the reference's own fixtures,
like the numpy oracle (``oracle/matcher_np.py``).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def _conv(sd, name, x):
    return F.conv1d(x, sd[name + ".weight"], sd[name + ".bias"])


def _linear_attention(q, k, v):
    """GATs_SuperGlue.py:88-99; q [B,64,4,Nq], k/v [B,64,4,Ns]."""
    eps = 1e-6
    q = F.elu(q) + 1
    k = F.elu(k) + 1
    v_length = v.size(3)
    v = v / v_length
    kv = torch.einsum("bdhm,bqhm->bqdh", k, v)
    z = 1 / (torch.einsum("bdhm,bdh->bhm", q, k.sum(3)) + eps)
    return torch.einsum("bdhm,bqdh,bhm->bqhm", q, kv, z) * v_length


def _propagation(sd, pre, x, source):
    """AttentionPropagation.forward (:130-132) with MultiHeadedAttention (:112-120)."""
    b = x.size(0)
    q = _conv(sd, pre + "attn.proj.0", x).view(b, 64, 4, -1)
    k = _conv(sd, pre + "attn.proj.1", source).view(b, 64, 4, -1)
    v = _conv(sd, pre + "attn.proj.2", source).view(b, 64, 4, -1)
    msg = _conv(sd, pre + "attn.merge", _linear_attention(q, k, v).reshape(b, 256, -1))
    h = _conv(sd, pre + "mlp.0", torch.cat([x, msg], dim=1))
    h = F.relu(F.instance_norm(h, eps=1e-5))
    return _conv(sd, pre + "mlp.3", h)


def _gat(sd, pre, h_2d, h_3d):
    """GraphAttentionLayer.forward (GATs.py:62-104): include_self, no linear transform."""
    W, a = sd[pre + "W"], sd[pre + "a"]
    b, n1, dim = h_3d.shape
    L = h_2d.size(1) // n1
    wh_2d = h_2d @ W
    wh_3d = h_3d @ W
    s2 = (wh_2d @ a[:dim]).view(b, n1, L, 1)
    s3 = wh_3d @ a[dim:]
    e = s3.unsqueeze(2) + torch.cat([s3.unsqueeze(2), s2], dim=2)
    att = torch.softmax(F.leaky_relu(e, 0.2), dim=2)
    hcat = torch.cat([h_3d.unsqueeze(2), h_2d.view(b, n1, L, dim)], dim=2)
    return F.elu(torch.einsum("bncd,bncq->bnq", att, hcat))


def to_torch(sd):
    return {k: torch.from_numpy(np.ascontiguousarray(v, np.float32)) for k, v in sd.items()}


@torch.no_grad()
def forward(sd, data, scale_factor=0.07, match_threshold=0.2):
    """GATsSuperGlue.forward on CPU tensors.  ``sd``: state dict of torch tensors (``to_torch``),
    ``data``: numpy arrays or tensors in the reference layout.  Returns (pred for batch 0,
    conf)."""
    t = {k: torch.as_tensor(v) for k, v in data.items()}
    d2 = t["descriptors2d_query"].float()
    d3 = t["descriptors3d_db"].float()
    db = t["descriptors2d_db"].float()
    for i, kind in enumerate(["GATs", "self", "cross"] * 4):
        pre = f"gnn.layers.{i}."
        if kind == "GATs":
            d3 = _gat(sd, pre, db.transpose(1, 2), d3.transpose(1, 2)).transpose(1, 2)
        elif kind == "cross":
            a, c = _propagation(sd, pre, d2, d3), _propagation(sd, pre, d3, d2)
            d2, d3 = d2 + a, d3 + c
        else:
            a, c = _propagation(sd, pre, d2, d2), _propagation(sd, pre, d3, d3)
            d2, d3 = d2 + a, d3 + c
    m2 = F.normalize(_conv(sd, "final_proj", d2), dim=1)
    m3 = F.normalize(_conv(sd, "final_proj", d3), dim=1)
    scores = torch.einsum("bdn,bdm->bnm", m2, m3) / scale_factor
    conf = F.softmax(scores, 1) * F.softmax(scores, 2)
    max0, max1 = conf.max(2), conf.max(1)
    idx0, idx1 = max0.indices, max1.indices
    mutual0 = torch.arange(idx0.size(1))[None] == idx1.gather(1, idx0)
    mutual1 = torch.arange(idx1.size(1))[None] == idx0.gather(1, idx1)
    zero = conf.new_tensor(0)
    ms0 = torch.where(mutual0, max0.values, zero)
    ms1 = torch.where(mutual1, ms0.gather(1, idx1), zero)
    valid0 = mutual0 & (ms0 > match_threshold)
    valid1 = mutual1 & valid0.gather(1, idx1)
    m0 = torch.where(valid0, idx0, idx0.new_tensor(-1))
    m1 = torch.where(valid1, idx1, idx1.new_tensor(-1))
    pred = {"matches0": m0[0].numpy(), "matches1": m1[0].numpy(),
            "matching_scores0": ms0[0].numpy(), "matching_scores1": ms1[0].numpy()}
    return pred, conf.numpy()
