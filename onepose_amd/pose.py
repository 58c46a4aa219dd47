"""Pose solve and pose error for the OnePose hot path, on libonepose_hip.

Drop-ins (same names, argument meaning and failure behaviour as the reference):

* ``ransac_PnP(K, pts_2d, pts_3d, scale=1)`` -- ``src/utils/eval_utils.py:18-42``: returns
  ``(pose [3,4], pose_homo [4,4], inliers [k,1] int32)``; on the reference's cv2.error path
  (fewer than 4 points) it prints ``CV ERROR`` and returns ``eye(4)[:3], eye(4), []``.
* ``query_pose_error(pose_pred, pose_gt)`` -- ``eval_utils.py:45-63``.
* ``Evaluator`` -- ``src/evaluators/cmd_evaluator.py:3-62`` (1/3/5 cm-deg rates).
* ``record_eval_result(out_dir, obj_name, seq_name, eval_result)`` -- ``eval_utils.py:7-15``.

Batched device APIs used by the pipeline (no host round trip per frame):
``select_correspondences``, ``ransac_pnp_batch``, ``pose_errors``.
"""
from __future__ import annotations

import os
from pathlib import Path

import numpy as np
import torch

from . import _lib

STATUS_OK, STATUS_TOO_FEW, STATUS_NO_MODEL = 0, 1, 2


def select_correspondences(matches0, kpts2d, kpts3d, scale=1.0):
    """Device version of ``inference.py:147-152`` for a batch: ``matches0 [B,N1] int64``,
    ``kpts2d [B,N1,2]``, ``kpts3d [B,N3,3]`` (or ``[N3,3]`` shared) -> compacted
    ``pts2d [B,N1,2]``, ``pts3d [B,N1,3]`` float32 (3D scaled by ``scale`` in float64 then
    rounded to float32, as solvePnPRansac sees them) and ``counts [B]`` int32."""
    lib = _lib.load()
    if kpts3d.dim() == 2:
        kpts3d = kpts3d[None]
    B, n1 = matches0.shape
    n3 = kpts3d.shape[1]
    kp2 = kpts2d.float().contiguous()
    kp3 = kpts3d.float()
    if kp3.shape[0] == 1 or kp3.stride(0) == 0:
        kp3_bs = 0
        kp3 = kp3[:1].contiguous()
    else:
        kp3 = kp3.contiguous()
        kp3_bs = n3 * 3
    dev = matches0.device
    p2 = torch.empty(B, n1, 2, dtype=torch.float32, device=dev)
    p3 = torch.empty(B, n1, 3, dtype=torch.float32, device=dev)
    counts = torch.empty(B, dtype=torch.int32, device=dev)
    _lib.check(lib.onepose_select_correspondences(
        matches0.contiguous().data_ptr(), kp2.data_ptr(), n1 * 2, kp3.data_ptr(), kp3_bs, B, n1, n3,
        float(scale), p2.data_ptr(), p3.data_ptr(), counts.data_ptr(), _lib.stream_ptr(dev)),
        "select_correspondences")
    return p2, p3, counts


def ransac_pnp_batch(pts2d, pts3d, counts, K, scale=1.0, reprojection_error=5.0,
                     iterations_count=10000, confidence=0.99, workspace=None):
    """Batched RANSAC-EPnP on the device.  ``pts2d [B,M,2]``, ``pts3d [B,M,3]`` float32
    (already scaled), ``counts [B]`` int32, ``K [B,3,3]`` or ``[3,3]`` float64.
    Returns ``pose34 [B,3,4]`` float64 (t divided by ``scale``), ``inlier_mask [B,M]`` uint8,
    ``n_inliers [B]``, ``status [B]``."""
    lib = _lib.load()
    B, M = pts2d.shape[0], pts2d.shape[1]
    dev = pts2d.device
    K = torch.as_tensor(K, dtype=torch.float64, device=dev)
    k_bs = 0 if K.dim() == 2 else 9
    K = K.contiguous()
    pose = torch.empty(B, 3, 4, dtype=torch.float64, device=dev)
    mask = torch.empty(B, M, dtype=torch.uint8, device=dev)
    n_in = torch.empty(B, dtype=torch.int32, device=dev)
    status = torch.empty(B, dtype=torch.int32, device=dev)
    ws_bytes = lib.onepose_pnp_workspace_bytes(B, M, int(iterations_count))
    if workspace is None or workspace.numel() < ws_bytes:
        workspace = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    _lib.check(lib.onepose_pnp_ransac(
        pts2d.contiguous().data_ptr(), pts3d.contiguous().data_ptr(), counts.data_ptr(), M,
        K.data_ptr(), k_bs, B, float(scale), float(reprojection_error), int(iterations_count),
        float(confidence), pose.data_ptr(), mask.data_ptr(), n_in.data_ptr(), status.data_ptr(),
        workspace.data_ptr(), ws_bytes, _lib.stream_ptr(dev)), "pnp_ransac")
    return pose, mask, n_in, status


def pose_errors(pose_pred, pose_gt):
    """Device cm/deg errors: ``pose_pred [B,3,4]``, ``pose_gt [B,3,4]`` or ``[3,4]`` float64
    -> ``(R_err_deg [B], t_err_cm [B], cmd [B,3] uint8 for 1/3/5 cm-deg)``."""
    lib = _lib.load()
    dev = pose_pred.device
    B = pose_pred.shape[0]
    gt = torch.as_tensor(pose_gt, dtype=torch.float64, device=dev)
    if gt.shape[-2] == 4:
        gt = gt[..., :3, :]
    gt_bs = 0 if gt.dim() == 2 else 12
    gt = gt.contiguous()
    r = torch.empty(B, dtype=torch.float64, device=dev)
    t = torch.empty(B, dtype=torch.float64, device=dev)
    cmd = torch.empty(B, 3, dtype=torch.uint8, device=dev)
    _lib.check(lib.onepose_pose_errors(pose_pred.contiguous().data_ptr(), gt.data_ptr(), gt_bs, B,
                                       r.data_ptr(), t.data_ptr(), cmd.data_ptr(),
                                       _lib.stream_ptr(dev)), "pose_errors")
    return r, t, cmd


def _default_device():
    if not torch.cuda.is_available():
        raise RuntimeError("onepose_amd.pose runs on a ROCm GPU only")
    return torch.device("cuda", torch.cuda.current_device())


def ransac_PnP(K, pts_2d, pts_3d, scale=1):
    """Drop-in for ``eval_utils.ransac_PnP`` (host numpy in, host numpy out)."""
    pts_2d = np.ascontiguousarray(np.asarray(pts_2d, dtype=np.float64)).reshape(-1, 2)
    pts_3d = np.ascontiguousarray(np.asarray(pts_3d, dtype=np.float64)).reshape(-1, 3)
    n = pts_2d.shape[0]
    if n < 4 or pts_3d.shape[0] != n:
        print("CV ERROR")
        return np.eye(4)[:3], np.eye(4), []
    dev = _default_device()
    p2 = torch.from_numpy(pts_2d.astype(np.float32)).to(dev)[None]
    p3 = torch.from_numpy((pts_3d * scale).astype(np.float32)).to(dev)[None]
    counts = torch.tensor([n], dtype=torch.int32, device=dev)
    pose, mask, n_in, status = ransac_pnp_batch(p2, p3, counts, np.asarray(K, np.float64),
                                                scale=float(scale))
    st = int(status.item())
    if st != STATUS_OK:   # cv2.solvePnPRansac returned False / raised: identity, no inliers
        return np.eye(4)[:3], np.eye(4), []
    pose = pose[0].cpu().numpy()
    pose_homo = np.concatenate([pose, np.array([[0, 0, 0, 1]])], axis=0)
    inliers = np.nonzero(mask[0].cpu().numpy())[0].astype(np.int32).reshape(-1, 1)
    return pose, pose_homo, inliers


def record_eval_result(out_dir, obj_name, seq_name, eval_result):
    """``eval_utils.record_eval_result``: one ``key: value`` line per summary entry in
    ``<out_dir>/<obj_name><seq_name>.txt`` (the directory is created)."""
    Path(out_dir).mkdir(exist_ok=True, parents=True)
    out_file = os.path.join(out_dir, obj_name + seq_name + ".txt")
    with open(out_file, "w") as f:
        for k, v in eval_result.items():
            f.write(f"{k}: {v}\n")
    return out_file


def query_pose_error(pose_pred, pose_gt):
    """``eval_utils.query_pose_error``: (angular deg, translation cm)."""
    pose_pred = np.asarray(pose_pred)
    pose_gt = np.asarray(pose_gt)
    if pose_pred.shape[0] == 4:
        pose_pred = pose_pred[:3]
    if pose_gt.shape[0] == 4:
        pose_gt = pose_gt[:3]
    translation_distance = np.linalg.norm(pose_pred[:, 3] - pose_gt[:, 3]) * 100
    trace = np.trace(pose_pred[:, :3] @ pose_gt[:, :3].T)
    trace = trace if trace <= 3 else 3
    angular_distance = np.rad2deg(np.arccos((trace - 1.0) / 2.0))
    return angular_distance, translation_distance


class Evaluator:
    """``cmd_evaluator.Evaluator``: accumulate 1/3/5 cm-deg hits, ``summarize()`` the rates."""

    def __init__(self):
        self.cmd1, self.cmd3, self.cmd5, self.cmd7, self.add = [], [], [], [], []

    def evaluate(self, pose_pred, pose_gt):
        if pose_pred is None:
            self.cmd5.append(False)
            self.cmd1.append(False)
            self.cmd3.append(False)
            self.cmd7.append(False)
            return
        pose_pred, pose_gt = np.asarray(pose_pred), np.asarray(pose_gt)
        if pose_pred.shape == (4, 4):
            pose_pred = pose_pred[:3, :4]
        if pose_gt.shape == (4, 4):
            pose_gt = pose_gt[:3, :4]
        ang, tr = query_pose_error(pose_pred, pose_gt)
        self.cmd1.append(tr < 1 and ang < 1)
        self.cmd3.append(tr < 3 and ang < 3)
        self.cmd5.append(tr < 5 and ang < 5)

    def evaluate_flags(self, cmd):
        """Accumulate device-computed 1/3/5 flags (``pose_errors``' ``cmd``, [B,3])."""
        cmd = np.asarray(cmd.cpu() if isinstance(cmd, torch.Tensor) else cmd).astype(bool)
        self.cmd1.extend(cmd[:, 0].tolist())
        self.cmd3.extend(cmd[:, 1].tolist())
        self.cmd5.extend(cmd[:, 2].tolist())

    def summarize(self):
        cmd1, cmd3, cmd5 = np.mean(self.cmd1), np.mean(self.cmd3), np.mean(self.cmd5)
        print("1 cm 1 degree metric: {}".format(cmd1))
        print("3 cm 3 degree metric: {}".format(cmd3))
        print("5 cm 5 degree metric: {}".format(cmd5))
        self.cmd1, self.cmd3, self.cmd5, self.cmd7 = [], [], [], []
        return {"cmd1": cmd1, "cmd3": cmd3, "cmd5": cmd5}
