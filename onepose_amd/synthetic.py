"""Seeded synthetic weights and scenes for the GATsSPG 2D-3D path.

There are no checkpoints or datasets in this environment, so every
test, fixture and benchmark is driven by the generators below.  They only use
``numpy.random.RandomState`` (legacy stream, version-stable) so fixtures made here
regenerate bit-identically on the GPU box.

* ``make_state_dict`` -- a ``GATsSuperGlue`` state dict with the reference's keys and
  shapes (``src/models/GATsSPG_architectures/GATs_SuperGlue.py:162-201``, ``GATs.py:50-53``).
  ``well_conditioned=True`` follows SURVEY.md §8c: ``final_proj`` orthogonal with zero
  bias and every ``mlp[-1].weight`` scaled by ``mlp_scale`` (0.01-0.05) so the GNN keeps
  descriptors close to their inputs and the matcher produces real matches.
* ``make_object`` -- one object's SfM cloud: 3D points, per-point collected 2D
  descriptors + ``idxs`` (the ``anno_3d_collect.npz`` / ``idxs.npy`` format,
  ``src/sfm/postprocess/feature_process.py:191-194,357-363``) and their averages
  (``anno_3d_average.npz``, ``feature_process.py:297-305``).
* ``make_frame`` -- one query frame of that object: GT pose, crop intrinsics, 2D keypoints
  (projected inliers + uniform outliers) and unit 2D descriptors, using the projection
  convention of ``src/utils/vis_utils.py:209-236`` (``K [R|t] X``).
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass

import numpy as np

DESC_DIM = 256
HEADS = 4
N_LAYERS = 12          # ['GATs', 'self', 'cross'] * 4  (GATs_SuperGlue.py:184)
KENC_LAYERS = (32, 64, 128)

DEFAULT_HPARAMS = {
    # configs/experiment/train_GATsSPG.yaml:44-60
    "descriptor_dim": 256,
    "keypoints_encoder": [32, 64, 128],
    "match_threshold": 0.2,
    "match_type": "softmax",
    "scale_factor": 0.07,
    "include_self": True,
    "with_linear_transform": False,
    "additional": False,
}


def layer_kind(i: int) -> str:
    return ("GATs", "self", "cross")[i % 3]


def _conv_default(rs, out_c, in_c):
    # torch.nn.Conv1d default init: kaiming_uniform(a=sqrt(5)) -> U(-1/sqrt(fan_in), +)
    bound = 1.0 / np.sqrt(in_c)
    w = rs.uniform(-bound, bound, size=(out_c, in_c, 1)).astype(np.float32)
    b = rs.uniform(-bound, bound, size=(out_c,)).astype(np.float32)
    return w, b


def _xavier_normal(rs, shape, gain=1.414):
    # GATs.py:50-53 -- nn.init.xavier_normal_(gain=1.414); fan_in = size(1), fan_out = size(0)
    fan_out, fan_in = shape[0], shape[1]
    std = gain * np.sqrt(2.0 / (fan_in + fan_out))
    return (rs.standard_normal(size=shape) * std).astype(np.float32)


def make_state_dict(seed: int = 0, well_conditioned: bool = True,
                    mlp_scale: float = 0.03) -> dict[str, np.ndarray]:
    """A full ``GATsSuperGlue`` state dict (5,674,401 parameters) as float32 numpy."""
    rs = np.random.RandomState(seed)
    sd: dict[str, np.ndarray] = {}
    sd["bin_score"] = np.array(1.0, dtype=np.float32)
    for name, inp in (("kenc_2d", 3), ("kenc_3d", 4)):
        chans = [inp, *KENC_LAYERS, DESC_DIM]
        for j in range(len(chans) - 1):
            w, b = _conv_default(rs, chans[j + 1], chans[j])
            if j == len(chans) - 2:
                b[:] = 0.0
            sd[f"{name}.encoder.{3 * j}.weight"] = w
            sd[f"{name}.encoder.{3 * j}.bias"] = b
    for i in range(N_LAYERS):
        p = f"gnn.layers.{i}"
        if layer_kind(i) == "GATs":
            sd[f"{p}.W"] = _xavier_normal(rs, (DESC_DIM, DESC_DIM))
            sd[f"{p}.a"] = _xavier_normal(rs, (2 * DESC_DIM, 1))
            continue
        w, b = _conv_default(rs, DESC_DIM, DESC_DIM)
        sd[f"{p}.attn.merge.weight"], sd[f"{p}.attn.merge.bias"] = w, b
        for j in range(3):
            w, b = _conv_default(rs, DESC_DIM, DESC_DIM)
            sd[f"{p}.attn.proj.{j}.weight"], sd[f"{p}.attn.proj.{j}.bias"] = w, b
        w, b = _conv_default(rs, 2 * DESC_DIM, 2 * DESC_DIM)
        sd[f"{p}.mlp.0.weight"], sd[f"{p}.mlp.0.bias"] = w, b
        w, b = _conv_default(rs, DESC_DIM, 2 * DESC_DIM)
        b[:] = 0.0                                    # GATs_SuperGlue.py:128
        if well_conditioned:
            w *= np.float32(mlp_scale)
        sd[f"{p}.mlp.3.weight"], sd[f"{p}.mlp.3.bias"] = w, b
    w, b = _conv_default(rs, DESC_DIM, DESC_DIM)
    if well_conditioned:
        q, r = np.linalg.qr(rs.standard_normal((DESC_DIM, DESC_DIM)))
        q = q * np.sign(np.diag(r))[None, :]
        w = q.astype(np.float32)[:, :, None]
        b = np.zeros(DESC_DIM, np.float32)
    sd["final_proj.weight"], sd["final_proj.bias"] = w, b
    return sd


def state_dict_sha(sd: dict[str, np.ndarray]) -> str:
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(np.ascontiguousarray(sd[k], dtype=np.float32).tobytes())
    return h.hexdigest()


def _unit_rows(x):
    return x / np.linalg.norm(x, axis=-1, keepdims=True)


@dataclass
class SynthObject:
    keypoints3d: np.ndarray        # [N3, 3] float32, metres, object frame
    desc3d_true: np.ndarray        # [N3, 256] unit "true" descriptor per 3D point
    clt_descriptors: np.ndarray    # [256, sum(idxs)] collected 2D descriptors (anno_3d_collect)
    clt_scores: np.ndarray         # [sum(idxs), 1]
    idxs: np.ndarray               # [N3] int64, observations per 3D point
    avg_descriptors: np.ndarray    # [256, N3] mean of each point's observations (anno_3d_average)
    avg_scores: np.ndarray         # [N3, 1]


def make_object(n3: int, seed: int = 0, noise: float = 0.3,
                min_obs: int = 2, max_obs: int = 12, box: float = 0.1) -> SynthObject:
    rs = np.random.RandomState(1000 + seed)
    kp3 = rs.uniform(-box, box, size=(n3, 3)).astype(np.float32)
    d3 = _unit_rows(rs.standard_normal((n3, DESC_DIM))).astype(np.float32)
    idxs = rs.randint(min_obs, max_obs + 1, size=n3).astype(np.int64)
    owner = np.repeat(np.arange(n3), idxs)
    u = _unit_rows(rs.standard_normal((owner.shape[0], DESC_DIM)))
    clt = _unit_rows(d3[owner] + noise * u).astype(np.float32)            # [sum, 256]
    clt_scores = rs.uniform(0.05, 1.0, size=(owner.shape[0], 1)).astype(np.float32)
    # mean_descriptors (feature_process.py:297-305): plain mean, NOT renormalised
    starts = np.concatenate([[0], np.cumsum(idxs)[:-1]])
    avg = np.add.reduceat(clt.astype(np.float64), starts, axis=0) / idxs[:, None]
    avg_s = np.add.reduceat(clt_scores.astype(np.float64), starts, axis=0) / idxs[:, None]
    return SynthObject(kp3, d3, np.ascontiguousarray(clt.T), clt_scores, idxs,
                       np.ascontiguousarray(avg.T.astype(np.float32)), avg_s.astype(np.float32))


def random_rotation(rs) -> np.ndarray:
    q = rs.standard_normal(4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)],
    ])


def crop_intrinsics(size: int = 512, f: float = 600.0) -> np.ndarray:
    return np.array([[f, 0.0, size / 2.0], [0.0, f, size / 2.0], [0.0, 0.0, 1.0]])


def project(K, pose34, pts):
    """vis_utils.reproj semantics: K [R|t] X, divided by depth."""
    cam = pts @ pose34[:, :3].T + pose34[:, 3]
    uv = cam @ K.T
    return uv[:, :2] / uv[:, 2:3]


@dataclass
class SynthFrame:
    keypoints2d: np.ndarray        # [N1, 2] float32 (x, y) pixels
    descriptors2d: np.ndarray      # [256, N1] float32 unit columns
    K: np.ndarray                  # [3, 3] float64
    pose_gt: np.ndarray            # [3, 4] float64, object -> camera, metres
    true_match: np.ndarray         # [N1] int64: 3D index for inlier rows, -1 for outliers


def make_frame(obj: SynthObject, n1: int, seed: int = 0, inlier_frac: float = 0.6,
               confuser_frac: float = 0.15, noise: float = 0.3, px_noise: float = 0.5,
               size: int = 512) -> SynthFrame:
    """Rows: ``inlier_frac`` projected 3D points (+``px_noise`` px) with noisy descriptors of
    their point; ``confuser_frac`` rows that carry a (different) 3D point's descriptor at a
    random pixel -- they match, but are gross outliers for PnP; the rest random."""
    rs = np.random.RandomState(2000 + seed)
    n3 = obj.keypoints3d.shape[0]
    n_in = min(int(round(inlier_frac * n1)), n3)
    n_cf = min(int(round(confuser_frac * n1)), n3 - n_in)
    n_out = n1 - n_in - n_cf
    R = random_rotation(rs)
    t = np.array([rs.uniform(-0.03, 0.03), rs.uniform(-0.03, 0.03), rs.uniform(0.35, 0.55)])
    pose = np.concatenate([R, t[:, None]], axis=1)
    K = crop_intrinsics(size)
    perm = rs.permutation(n3)
    pts, cpts = perm[:n_in], perm[n_in:n_in + n_cf]
    uv_in = project(K, pose, obj.keypoints3d[pts].astype(np.float64))
    uv_in += rs.normal(0.0, px_noise, size=uv_in.shape)
    uv_rest = rs.uniform(0, size, size=(n_cf + n_out, 2))
    d_in = _unit_rows(obj.desc3d_true[pts] + noise * _unit_rows(rs.standard_normal((n_in, DESC_DIM))))
    d_cf = _unit_rows(obj.desc3d_true[cpts] + noise * _unit_rows(rs.standard_normal((n_cf, DESC_DIM))))
    d_out = _unit_rows(rs.standard_normal((n_out, DESC_DIM)))
    kp = np.concatenate([uv_in, uv_rest]).astype(np.float32)
    desc = np.concatenate([d_in, d_cf, d_out]).astype(np.float32)
    truth = np.concatenate([pts, -np.ones(n_cf + n_out, np.int64)])
    order = rs.permutation(n1)
    return SynthFrame(kp[order], np.ascontiguousarray(desc[order].T), K, pose, truth[order])


def make_matcher_inputs(n1: int, n3: int, num_leaf: int = 8, seed: int = 0, batch: int = 1,
                        frame_ids=None):
    """Matcher inputs in the reference layout (GATs_SuperGlue.py:209-217), numpy float32.

    Leaves come from the build's own ``build_features3d_leaves`` restatement with a
    numpy RNG seeded here, as ``inference.py:113-130`` does after ``seed_everything``.
    Frame b of the object is ``make_frame(obj, n1, seed * 131 + b)``; ``frame_ids`` picks
    which frames of that one sequence to return (default ``range(batch)``), so a rank of a
    frame-sharded run builds exactly its slice of one global batch (distributed.frame_shard).
    """
    from .data_utils import build_features3d_leaves, pad_features3d_random
    obj = make_object(n3, seed)
    np.random.seed(12345 + seed)
    avg, _ = pad_features3d_random(obj.avg_descriptors, obj.avg_scores, n3)
    leaves, _ = build_features3d_leaves(obj.clt_descriptors, obj.clt_scores, obj.idxs, n3, num_leaf)
    avg, leaves = avg.numpy(), leaves.numpy()
    ids = list(range(batch)) if frame_ids is None else list(frame_ids)
    batch = len(ids)
    frames = [make_frame(obj, n1, seed * 131 + b) for b in ids]
    return {
        "keypoints2d": np.stack([f.keypoints2d for f in frames]),
        "keypoints3d": np.broadcast_to(obj.keypoints3d[None], (batch, n3, 3)).copy(),
        "descriptors2d_query": np.stack([f.descriptors2d for f in frames]),
        "descriptors3d_db": np.broadcast_to(avg[None], (batch,) + avg.shape).copy(),
        "descriptors2d_db": np.broadcast_to(leaves[None], (batch,) + leaves.shape).copy(),
    }, obj, frames



def make_frame_bank(n1: int, n3: int, steps: int, batch: int = 1, seed: int = 0, world: int = 1,
                    rank: int = 0):
    """Per-step query inputs of one object's sequence, for a bank of ``steps`` steps of
    ``batch`` frames on this rank: arrays [steps, batch, ...] (keypoints2d, descriptors2d_query
    in the reference's [256, n1] layout, K, pose_gt) and the global frame ids [steps, batch].
    Step j of the sequence holds global frames [j * world * batch, (j + 1) * world * batch),
    sharded contiguously over ranks (distributed.frame_shard), so rank r's frame (j, i) is
    global frame (j * world + r) * batch + i -- frame g is ``make_frame(obj, n1, seed * 131 +
    g)``, the same frames make_matcher_inputs(frame_ids=...) builds.  The object itself is not
    copied per frame (make_matcher_inputs broadcasts it over the batch)."""
    obj = make_object(n3, seed)
    gid = np.array([[(j * world + rank) * batch + i for i in range(batch)] for j in range(steps)],
                   np.int64)
    frames = [[make_frame(obj, n1, seed * 131 + int(g)) for g in row] for row in gid]
    return {
        "keypoints2d": np.stack([np.stack([f.keypoints2d for f in r]) for r in frames]),
        "descriptors2d_query": np.stack([np.stack([f.descriptors2d for f in r]) for r in frames]),
        "K": np.stack([np.stack([f.K for f in r]) for r in frames]),
        "pose_gt": np.stack([np.stack([f.pose_gt for f in r]) for r in frames]),
        "frame_id": gid,
    }

# ------------------------------------------------------------------ SuperPoint
SUPERPOINT_LAYERS = [   # (name, c_in, c_out, kernel)  superpoint.py:147-162
    ("conv1a", 1, 64, 3), ("conv1b", 64, 64, 3), ("conv2a", 64, 64, 3), ("conv2b", 64, 64, 3),
    ("conv3a", 64, 128, 3), ("conv3b", 128, 128, 3), ("conv4a", 128, 128, 3),
    ("conv4b", 128, 128, 3), ("convPa", 128, 256, 3), ("convPb", 256, 65, 1),
    ("convDa", 128, 256, 3), ("convDb", 256, 256, 1)]

# the reference extraction config (extract_features.py:19-24); note 'keypoints_threshold'
# is not a key SuperPoint reads, so its default keypoint_threshold 0.005 applies
SUPERPOINT_CONF = {"descriptor_dim": 256, "nms_radius": 3, "max_keypoints": 4096,
                   "keypoints_threshold": 0.6}


def superpoint_state_dict(seed: int = 0) -> dict[str, np.ndarray]:
    """Random SuperPoint weights (numpy RandomState, version-stable): He-uniform convs,
    small biases.  The trained weights (superpoint_v1.pth) are not available offline."""
    rs = np.random.RandomState(9000 + seed)
    sd = {}
    for name, cin, cout, k in SUPERPOINT_LAYERS:
        bound = np.sqrt(6.0 / (cin * k * k))
        sd[f"{name}.weight"] = rs.uniform(-bound, bound, (cout, cin, k, k)).astype(np.float32)
        sd[f"{name}.bias"] = rs.uniform(-0.05, 0.05, cout).astype(np.float32)
    return sd


def superpoint_image(h: int, w: int, seed: int = 0) -> np.ndarray:
    """A grayscale test image in [0, 1] ([h, w] float32): smooth blobs, edges and texture,
    so the detector finds distinct local maxima."""
    rs = np.random.RandomState(7000 + seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    img = np.zeros((h, w))
    for _ in range(24):
        cy, cx = rs.uniform(0, h), rs.uniform(0, w)
        s = rs.uniform(2.0, 9.0)
        img += rs.uniform(-1, 1) * np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * s * s))
    for _ in range(6):
        a, b, c = rs.uniform(-1, 1, 3)
        img += 0.3 * (a * (yy - h / 2) + b * (xx - w / 2) + c * h > 0)
    img += 0.05 * rs.randn(h, w)
    img = (img - img.min()) / (img.max() - img.min())
    return img.astype(np.float32)
