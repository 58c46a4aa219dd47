"""``inference.py``-compatible driver on the HIP engine (reference ``inference.py:17-200``).

Same inputs (an object's SfM annotation directory, a sequence directory of cropped images
with per-image ``intrin_ba`` / ``poses_ba`` text files, a matcher checkpoint, a keypoint
extractor) and the same per-frame steps and outputs (cm/deg evaluator summary). What
changes against the reference loop:

* the object's tensors go to the GPU once per object; ``pack_data`` re-uploads them every
  frame (``inference.py:80-94``);
* the matcher is ``onepose_amd.matcher.GATsSuperGlue`` (C-ABI, HIP), the pose solve
  ``onepose_amd.pose.ransac_PnP`` (HIP RANSAC-EPnP), the evaluator ``onepose_amd.pose.Evaluator``;
* the extractor is any callable ``image [1,1,H,W] -> {'keypoints', 'descriptors', ...}``.
  The reference's SuperPoint module is one; this repository's GPU backbone is §8f's next row.

Frames keep their own keypoint count (the detector thresholds at 0.6,
``extract_features.py:19-24``), so each frame runs at its true size: padding would change
the matcher's attention and InstanceNorm results. For fixed-size streams, ``FramePipeline``
is the graph-replayed throughput path.
"""
from __future__ import annotations

import glob
import os
import re

import numpy as np
import torch

from . import data_utils, pose
from .matcher import GATsSuperGlue, from_state_dict

REFERENCE_SEED = 12345   # inference.py:14  seed_everything(12345)


# ------------------------------------------------------------------ paths (path_utils.py)
def _swap_dir(path: str, old: str, new: str) -> str:
    """Replace the ``old`` directory component (either separator) by ``new``."""
    return re.sub(r"([\\/])" + re.escape(old) + r"([\\/])", lambda m: m.group(1) + new + m.group(2),
                  path, count=1)


def get_gt_pose_path_by_color(color_path: str, det_type: str = "GT_box") -> str:
    """path_utils.py:22-31 (the reference spells the separators as backslashes)."""
    src = {"GT_box": "color", "feature_matching": "color_det"}.get(det_type)
    if src is None:
        raise NotImplementedError(det_type)
    return _swap_dir(color_path, src, "poses_ba").replace(".png", ".txt")


def get_intrin_path_by_color(color_path: str, det_type: str = "GT_box") -> str:
    """path_utils.py:43-52."""
    if det_type == "GT_box":
        return _swap_dir(color_path, "color", "intrin_ba").replace(".png", ".txt")
    if det_type == "feature_matching":
        return _swap_dir(color_path, "color_det", "intrin_det").replace(".png", ".txt")
    raise NotImplementedError(det_type)


def get_default_paths(data_dir: str, sfm_model_dir: str, detection: str = "superpoint",
                      matching: str = "superglue", object_detect_mode: str = "GT_box"):
    """inference.py:17-47: (image list, paths). Images are sorted (the reference takes glob
    order)."""
    anno_dir = os.path.join(sfm_model_dir, f"outputs_{detection}_{matching}", "anno")
    if object_detect_mode == "GT_box":
        color_dir = os.path.join(data_dir, "color")
    elif object_detect_mode == "feature_matching":
        color_dir = os.path.join(data_dir, "color_det")
        if not os.path.exists(color_dir):
            raise FileNotFoundError("color_det directory not found: run the 2D object detector "
                                    "first (reference README)")
    else:
        raise NotImplementedError(object_detect_mode)
    img_lists = sorted(glob.glob(color_dir + "/*.png"))
    paths = {"data_dir": data_dir, "sfm_model_dir": sfm_model_dir, "anno_dir": anno_dir,
             "avg_anno_3d_path": os.path.join(anno_dir, "anno_3d_average.npz"),
             "clt_anno_3d_path": os.path.join(anno_dir, "anno_3d_collect.npz"),
             "idxs_path": os.path.join(anno_dir, "idxs.npy"),
             "intrin_full_path": os.path.join(data_dir, "intrinsics.txt")}
    return img_lists, paths


# ------------------------------------------------------------------ model and object
def load_matcher(model_path: str | None = None, state_dict=None, hparams=None) -> GATsSuperGlue:
    """The matcher of a ``LitModelGATsSPG`` checkpoint (``inference.py:50-59``).

    The checkpoint is read with ``torch.load(weights_only=True)``: only tensors and plain
    containers are accepted, nothing in the file is executed. ``state_dict['matcher.*']``
    holds the weights; ``hyper_parameters`` (flat, ``GATsSPG_lightning_model.py:17-21``)
    the matcher config unless ``hparams`` is given. A checkpoint whose hyper-parameters need
    unpickling of foreign classes is refused by the safe loader; pass ``state_dict`` +
    ``hparams`` explicitly then."""
    if state_dict is None:
        ckpt = torch.load(model_path, map_location="cpu", weights_only=True)
        sd = ckpt.get("state_dict", ckpt)
        if hparams is None and isinstance(ckpt.get("hyper_parameters"), dict):
            hparams = dict(ckpt["hyper_parameters"])
    else:
        sd = state_dict
    if any(k.startswith("matcher.") for k in sd):
        sd = {k[len("matcher."):]: v for k, v in sd.items() if k.startswith("matcher.")}
    if hparams is not None:
        from .synthetic import DEFAULT_HPARAMS
        hparams = {**DEFAULT_HPARAMS, **{k: hparams[k] for k in DEFAULT_HPARAMS if k in hparams}}
    return from_state_dict(sd, hparams)


class OnePoseObject:
    """One object's SfM model on the device (``inference.py:108-130``, uploaded once)."""

    def __init__(self, keypoints3d, descriptors3d, leaves, device):
        f32 = dict(dtype=torch.float32, device=device)
        self.keypoints3d = torch.as_tensor(keypoints3d).to(**f32).contiguous()   # [N3, 3]
        self.descriptors3d = torch.as_tensor(descriptors3d).to(**f32).contiguous()  # [256, N3]
        self.leaves = torch.as_tensor(leaves).to(**f32).contiguous()             # [256, N3*L]
        self.num_leaf = self.leaves.shape[1] // self.keypoints3d.shape[0]

    @classmethod
    def from_anno_dir(cls, anno_dir: str, num_leaf: int = 8, device="cuda"):
        """Reads the three annotation files and builds padded / leaf descriptors with the
        global numpy stream, as the reference does after ``seed_everything``."""
        kp3, avg, leaves = data_utils.load_object_annotations(anno_dir, num_leaf)
        return cls(kp3, avg, leaves, device)


# ------------------------------------------------------------------ per frame
def load_image(path: str, grayscale: bool = True):
    """NormalizedDataset.__getitem__ (normalized_dataset.py:22-41): float32 / 255,
    [1,H,W] grayscale or [3,H,W]; returns (image, (H, W))."""
    from PIL import Image
    img = Image.open(path)
    img = np.asarray(img.convert("L" if grayscale else "RGB"), dtype=np.float32)
    img = img[None] if grayscale else img[..., ::-1].transpose(2, 0, 1)   # cv2 reads BGR
    return np.ascontiguousarray(img / 255.0, dtype=np.float32), img.shape[-2:]


def match_and_pose(matcher: GATsSuperGlue, obj: OnePoseObject, keypoints2d, descriptors2d, K,
                   scale: float = 1000.0):
    """One frame of ``inference.py:143-155``: matcher -> valid matches -> RANSAC-EPnP.
    Returns (pose [3,4], pose_homo [4,4], inliers, mkpts2d, mkpts3d, mconf)."""
    dev = obj.keypoints3d.device
    kp2 = torch.as_tensor(np.asarray(keypoints2d, np.float32), device=dev)
    d2 = torch.as_tensor(np.asarray(descriptors2d, np.float32), device=dev)
    inp = {"keypoints2d": kp2[None], "keypoints3d": obj.keypoints3d[None],
           "descriptors2d_query": d2[None], "descriptors3d_db": obj.descriptors3d[None],
           "descriptors2d_db": obj.leaves[None]}
    with torch.no_grad():
        pred, _ = matcher(inp)
    matches = pred["matches0"].cpu().numpy()
    valid = matches > -1
    kpts2d = np.asarray(keypoints2d)
    kpts3d = obj.keypoints3d.cpu().numpy()
    conf = pred["matching_scores0"].cpu().numpy()
    mk2, mk3, mconf = kpts2d[valid], kpts3d[matches[valid]], conf[valid]
    pose_pred, pose_homo, inliers = pose.ransac_PnP(K, mk2, mk3, scale=scale)
    return pose_pred, pose_homo, inliers, mk2, mk3, mconf


def run_frames(matcher: GATsSuperGlue, obj: OnePoseObject, frames, scale: float = 1000.0):
    """The evaluation loop over precomputed detections: each frame a dict with keypoints2d
    [n,2], descriptors2d [256,n], K [3,3], pose_gt [3,4] or [4,4]. Returns (summary,
    per-frame [(pose_pred, n_inliers)])."""
    ev = pose.Evaluator()
    out = []
    for f in frames:
        p, _, inl, *_ = match_and_pose(matcher, obj, f["keypoints2d"], f["descriptors2d"], f["K"],
                                       scale)
        ev.evaluate(p, f["pose_gt"])
        out.append((p, len(inl)))
    return ev.summarize(), out


def inference_core(matcher: GATsSuperGlue, extractor, seq_dir: str, sfm_model_dir: str,
                   num_leaf: int = 8, object_detect_mode: str = "GT_box", device="cuda",
                   detection: str = "superpoint", matching: str = "superglue"):
    """inference.py:97-177 for one sequence (no visualisation): returns the evaluator summary.
    ``extractor(image [1,1,H,W] on device)`` returns the reference SuperPoint's output dict
    (keys 'keypoints' [1][n,2], 'descriptors' [1][256,n])."""
    img_lists, paths = get_default_paths(seq_dir, sfm_model_dir, detection, matching,
                                         object_detect_mode)
    obj = OnePoseObject.from_anno_dir(paths["anno_dir"], num_leaf, device)
    ev = pose.Evaluator()
    for img_path in img_lists:
        img, _ = load_image(img_path)
        det = extractor(torch.from_numpy(img)[None].to(device))
        det = {k: (v[0].detach().cpu().numpy() if torch.is_tensor(v[0]) else np.asarray(v[0]))
               for k, v in det.items()}
        K = np.loadtxt(get_intrin_path_by_color(img_path, object_detect_mode))
        p, _, _, *_ = match_and_pose(matcher, obj, det["keypoints"], det["descriptors"], K)
        ev.evaluate(p, np.loadtxt(get_gt_pose_path_by_color(img_path, object_detect_mode)))
    return ev.summarize()


def seed_reference_stream(seed: int = REFERENCE_SEED):
    """The numpy / torch seeding ``inference.py:14`` performs at import."""
    np.random.seed(seed)
    torch.manual_seed(seed)
