"""ORACLE -- test infrastructure only.  Never imported by the product path.

The N3-sharded GATsSPG forward (onepose_match_sharded, include/onepose_hip.h) restated in
numpy, all shards simulated in one process: the 3D points are split with the library's rule
(start_r = floor(n3 * r / world)), every shard keeps the whole 2D side, and the quantities
that cross shards are formed exactly as the device merges them --
  * per attention layer: KV = sum_r KV_r and sum phi(k) = sum_r (linear attention over a
    3D source, GATs_SuperGlue.py:88-99, with v / n3_total and Ns = n3_total);
  * per attention layer: the 3D side's InstanceNorm (:135-147) from the shards' (n, mean,
    M2), Chan-merged in rank order;
  * dual softmax (:251-253): row max / sum over every shard's columns;
  * mutual NN (:256-267): on the assembled full-width conf.
Its agreement with matcher_np.forward (tests/test_sharded_oracle.py) shows the exchanged
partials are sufficient and exact up to summation order."""
from __future__ import annotations

import numpy as np

from .matcher_np import (F32, _conv1x1, _elu, _normalize, gat_layer, layer_params,
                         match_head)


def shard_range(n3, world, rank):
    start = n3 * rank // world
    return start, n3 * (rank + 1) // world - start


def _proj(p, i, x):
    b = x.shape[0]
    return _conv1x1(p[f"attn.proj.{i}.weight"], p[f"attn.proj.{i}.bias"], x).reshape(b, 64, 4, -1)


def kv_partial(p, source, n_total):
    """This shard's share of KV and sum phi(k) (linear_attention with v / n_total)."""
    k = _elu(_proj(p, 1, source)) + F32(1)
    v = _proj(p, 2, source) / F32(n_total)
    kv = np.einsum("bdhm,bqhm->bqdh", k, v, optimize=True)
    return kv, k.sum(3)


def message_hidden(p, x, kv, ksum, n_total):
    """Query side of the attention + merge conv + mlp.0 (pre-norm hidden), given the
    source's (merged) KV / sum phi(k)."""
    b = x.shape[0]
    q = _elu(_proj(p, 0, x)) + F32(1)
    z = F32(1) / (np.einsum("bdhm,bdh->bhm", q, ksum, optimize=True) + F32(1e-6))
    msg = (np.einsum("bdhm,bqdh->bqhm", q, kv, optimize=True) * z[:, None] * F32(n_total))
    msg = _conv1x1(p["attn.merge.weight"], p["attn.merge.bias"], msg.astype(F32).reshape(b, 256, -1))
    return _conv1x1(p["mlp.0.weight"], p["mlp.0.bias"], np.concatenate([x, msg], axis=1))


def moments(h):
    """(n, mean, M2) per (b, c) of a shard's hidden [B,512,N], float64."""
    h64 = h.astype(np.float64)
    mean = h64.mean(axis=2)
    return h.shape[2], mean, ((h64 - mean[..., None]) ** 2).sum(axis=2)


def chan_merge(parts):
    """Merge (n, mean, M2) in order -> (mean, biased var)."""
    n, mean, m2 = 0, 0.0, 0.0
    for nb, mb, m2b in parts:
        nn = n + nb
        delta = mb - mean
        mean = mean + delta * (nb / nn)
        m2 = m2 + m2b + delta * delta * (n * nb / nn)
        n = nn
    return mean, m2 / n


def finish(p, h, mean, var):
    hn = ((h.astype(np.float64) - mean[..., None]) / np.sqrt(var[..., None] + 1e-5)).astype(F32)
    return _conv1x1(p["mlp.3.weight"], p["mlp.3.bias"], np.maximum(hn, F32(0)))


def forward(sd, data, world, scale_factor=0.07, match_threshold=0.2):
    """Sharded GATsSuperGlue forward; returns (m0, m1, ms0, ms1, conf) over all batches."""
    d2 = np.asarray(data["descriptors2d_query"], F32)
    d3 = np.asarray(data["descriptors3d_db"], F32)
    db = np.asarray(data["descriptors2d_db"], F32)
    n3 = d3.shape[2]
    L = db.shape[2] // n3
    ranges = [shard_range(n3, world, r) for r in range(world)]
    s3 = [d3[:, :, s:s + c] for s, c in ranges]
    lv = [db[:, :, s * L:(s + c) * L] for s, c in ranges]
    for i, name in enumerate(["GATs", "self", "cross"] * 4):
        p = layer_params(sd, i)
        if name == "GATs":
            s3 = [np.ascontiguousarray(gat_layer(p, l.transpose(0, 2, 1), x.transpose(0, 2, 1))
                                       .transpose(0, 2, 1)) for x, l in zip(s3, lv)]
            continue
        n1 = d2.shape[2]
        parts = [kv_partial(p, x, n3) for x in s3]          # the 3D side as a source
        kv3, ks3 = sum(q[0] for q in parts), sum(q[1] for q in parts)
        if name == "self":
            kv2, ks2 = kv_partial(p, d2, n1)
            h2 = message_hidden(p, d2, kv2, ks2, n1)
            h3 = [message_hidden(p, x, kv3, ks3, n3) for x in s3]
        else:
            kv2, ks2 = kv_partial(p, d2, n1)
            h2 = message_hidden(p, d2, kv3, ks3, n3)
            h3 = [message_hidden(p, x, kv2, ks2, n1) for x in s3]
        m2, v2 = chan_merge([moments(h2)])
        m3, v3 = chan_merge([moments(h) for h in h3])
        d2 = d2 + finish(p, h2, m2, v2)
        s3 = [x + finish(p, h, m3, v3) for x, h in zip(s3, h3)]
    f = (sd["final_proj.weight"], sd["final_proj.bias"])
    f2 = _normalize(_conv1x1(*f, d2), 1)
    f3 = [_normalize(_conv1x1(*f, x), 1) for x in s3]
    sc = [(np.einsum("bdn,bdm->bnm", f2, x, optimize=True) / F32(scale_factor)).astype(F32)
          for x in f3]
    # row softmax (over every shard's columns) from per-shard (max, sum)
    rmax = [s.max(axis=2) for s in sc]
    rsum = [np.exp(s - m[..., None]).sum(axis=2) for s, m in zip(sc, rmax)]
    M = np.max(np.stack(rmax), axis=0)
    S = sum(ss * np.exp(m - M) for ss, m in zip(rsum, rmax))
    conf = []
    for s in sc:
        col = np.exp(s - s.max(axis=1, keepdims=True))
        col = col / col.sum(axis=1, keepdims=True)
        row = np.exp(s - M[..., None]) / S[..., None]
        conf.append((col * row).astype(F32))
    conf = np.concatenate(conf, axis=2)
    return _mutual(conf, match_threshold)


def _mutual(conf, thr):
    idx0, idx1 = conf.argmax(axis=2), conf.argmax(axis=1)
    max0 = np.take_along_axis(conf, idx0[:, :, None], 2)[:, :, 0]
    n1, n3 = conf.shape[1], conf.shape[2]
    mutual0 = np.arange(n1)[None] == np.take_along_axis(idx1, idx0, 1)
    mutual1 = np.arange(n3)[None] == np.take_along_axis(idx0, idx1, 1)
    ms0 = np.where(mutual0, max0, F32(0)).astype(F32)
    ms1 = np.where(mutual1, np.take_along_axis(ms0, idx1, 1), F32(0)).astype(F32)
    valid0 = mutual0 & (ms0 > thr)
    valid1 = mutual1 & np.take_along_axis(valid0, idx1, 1)
    return (np.where(valid0, idx0, -1).astype(np.int64), np.where(valid1, idx1, -1).astype(np.int64),
            ms0, ms1, conf)


__all__ = ["forward", "shard_range", "match_head"]
