"""Per-object 3D packing (host side, once per object).

Mirrors the reference's object setup so a caller of ``src.utils.data_utils`` finds the
same functions with the same argument meaning and the same numpy-RNG consumption:

* ``pad_features3d_random``   -- ``src/utils/data_utils.py:143-160``
* ``build_features3d_leaves`` -- ``src/utils/data_utils.py:163-205``
* ``mean_descriptors`` / ``mean_scores`` -- ``src/sfm/postprocess/feature_process.py:297-317``
* ``load_object_annotations`` -- the on-disk format read by ``inference.py:113-130``
  (``anno_3d_average.npz``, ``anno_3d_collect.npz``, ``idxs.npy``; written by
  ``feature_process.py:191-194,357-363``).

This runs once per object, so it stays on the host like the reference's; the per-frame
work that consumes its output runs in HIP (see ``onepose_amd.matcher``).  The leaf
gather is vectorised, but the RNG is consumed exactly as the reference's per-point loop
does (one ``np.random.permutation`` per 3D point, in point order), so a run seeded like
``inference.py:13-14`` yields the same leaves.
"""
from __future__ import annotations

import os

import numpy as np
import torch


def _as_tensor(x):
    return x if isinstance(x, torch.Tensor) else torch.Tensor(np.asarray(x))


def pad_features3d_random(descriptors, scores, n_target_shape):
    """Pad (with ones / zero scores) or truncate the averaged 3D features to ``n_target_shape``."""
    descriptors = _as_tensor(descriptors)
    scores = _as_tensor(scores)
    dim = descriptors.shape[0]
    n_pad = n_target_shape - descriptors.shape[1]
    if n_pad < 0:
        return descriptors[:, :n_target_shape], scores[:n_target_shape, :]
    descriptors = torch.cat([descriptors, torch.ones(dim, n_pad)], dim=-1)
    scores = torch.cat([scores, torch.zeros(n_pad, 1)], dim=0)
    return descriptors, scores


def leaf_indices(idxs, num_leaf, dustbin_id, rng=None):
    """Column index of every leaf, ``[len(idxs) * num_leaf]`` int64.

    Per 3D point: its observations shuffled, padded with the dustbin column when there
    are fewer than ``num_leaf``, or the first ``num_leaf`` of a shuffle otherwise.
    """
    perm = (rng or np.random).permutation
    idxs = np.asarray(idxs).reshape(-1)
    upper = np.cumsum(idxs, axis=0)
    lower = np.insert(upper[:-1], 0, 0)
    out = np.empty((idxs.shape[0], num_leaf), dtype=np.int64)
    for p, (start, end) in enumerate(zip(lower, upper)):
        n = int(end - start)
        if num_leaf > n:
            cand = np.concatenate([np.arange(start, end), np.full(num_leaf - n, dustbin_id)])
            out[p] = perm(cand)
        else:
            out[p] = perm(np.arange(start, end))[:num_leaf]
    return out.reshape(-1)


def build_features3d_leaves(descriptors, scores, idxs, n_target_shape, num_leaf):
    """Gather ``num_leaf`` observation descriptors per 3D point -> ``[dim, n_target*num_leaf]``.

    The dustbin leaf is a column of ones (norm 16, not unit), as in the reference.
    """
    descriptors = _as_tensor(descriptors)
    scores = _as_tensor(scores)
    dim = descriptors.shape[0]
    orig_num = np.asarray(idxs).shape[0]
    n_pad = n_target_shape - orig_num
    desc_db = torch.cat([descriptors, torch.ones(dim, 1)], dim=1)
    scores_db = torch.cat([scores, torch.zeros(1, 1)], dim=0)
    cols = torch.from_numpy(leaf_indices(idxs, num_leaf, desc_db.shape[1] - 1))
    desc = desc_db[:, cols]
    sc = scores_db[cols, :]
    if n_pad < 0:
        return desc[:, :num_leaf * n_target_shape], sc[:num_leaf * n_target_shape, :]
    desc = torch.cat([desc, torch.ones(dim, n_pad * num_leaf)], dim=-1)
    sc = torch.cat([sc, torch.zeros(n_pad * num_leaf, 1)], dim=0)
    return desc, sc


def _segment_mean(values, idxs):
    idxs = np.asarray(idxs).reshape(-1)
    starts = np.insert(np.cumsum(idxs)[:-1], 0, 0)
    return np.stack([np.mean(values[s:s + n], axis=0) for s, n in zip(starts, idxs)])


def mean_descriptors(descriptors, idxs):
    """Average of each 3D point's observation descriptors ``[sum(idxs), dim] -> [N3, dim]``."""
    return _segment_mean(np.asarray(descriptors), idxs)


def mean_scores(scores, idxs):
    return _segment_mean(np.asarray(scores), idxs)


def load_object_annotations(anno_dir, num_leaf=8, max_num_kp3d=None):
    """Read one object's SfM annotations the way ``inference.py:113-130`` does.

    Returns ``(keypoints3d [N3,3], avg_descriptors [256,N3], leaf_descriptors [256,N3*L])``
    as float32 torch tensors on the CPU.
    """
    avg = np.load(os.path.join(anno_dir, "anno_3d_average.npz"))
    clt = np.load(os.path.join(anno_dir, "anno_3d_collect.npz"))
    idxs = np.load(os.path.join(anno_dir, "idxs.npy"))
    keypoints3d = torch.Tensor(clt["keypoints3d"])
    num_3d = keypoints3d.shape[0]
    avg_desc, _ = pad_features3d_random(avg["descriptors3d"], avg["scores3d"], num_3d)
    leaves, _ = build_features3d_leaves(clt["descriptors3d"], clt["scores3d"], idxs, num_3d, num_leaf)
    return keypoints3d, avg_desc, leaves


def save_object_annotations(anno_dir, keypoints3d, clt_descriptors, clt_scores, idxs):
    """Write the three files in the reference layout (``feature_process.py:191-194,357-363``):
    ``clt_descriptors`` [dim, sum(idxs)] as stored in ``anno_3d_collect.npz``.  The means are
    taken over the point-major [sum(idxs), dim] copy the reference averages (``get_kpt_ann``'s
    ``filter_descriptors``), so the summation order and the bits are the reference's."""
    os.makedirs(anno_dir, exist_ok=True)
    clt_descriptors = np.asarray(clt_descriptors)           # [dim, sum(idxs)]
    avg_d = mean_descriptors(np.ascontiguousarray(clt_descriptors.T), idxs)   # [N3, dim]
    avg_s = mean_scores(np.asarray(clt_scores), idxs)
    np.savez(os.path.join(anno_dir, "anno_3d_average.npz"), keypoints3d=keypoints3d,
             descriptors3d=avg_d.T, scores3d=avg_s)
    np.savez(os.path.join(anno_dir, "anno_3d_collect.npz"), keypoints3d=keypoints3d,
             descriptors3d=clt_descriptors, scores3d=clt_scores)
    np.save(os.path.join(anno_dir, "idxs.npy"), np.asarray(idxs))
