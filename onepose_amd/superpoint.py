"""SuperPoint keypoint detector + descriptor on libonepose_hip.

``SuperPoint(config)`` mirrors ``src/models/extractors/SuperPoint/superpoint.py:119-243``:
same ``default_config``, same parameter names (``conv1a.weight`` ... ``convDb.bias``), same
``forward(image [B,1,H,W]) -> {'keypoints': [n,2] (x,y), 'scores': [n], 'descriptors':
[256,n]}`` per image, same keypoint order.  The whole network, NMS, selection and sampling
run as HIP kernels (``onepose_superpoint``); ``detect_raw`` returns the fixed-capacity device
tensors without a host sync, for pipelines.  Image sides must be multiples of 8 (the
reference's OnePose crops are 512x512); other sizes raise.

``sample_descriptors(keypoints, descriptors, s=8)`` is the drop-in for
``src/models/extractors/SuperPoint/superpoint.py:95-113``: bilinear interpolation of the
dense descriptor map at the keypoints (zero padding), then L2 normalisation over channels.
``align_corners`` defaults to the reference's own rule -- ``int(torch.__version__[2]) > 2``
(superpoint.py:108), i.e. True on the pinned torch 1.8 and False on torch 2.x -- and can be
forced either way.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib


# src/sfm/extract_features.py:7-26, as the reference writes it. The 'keypoints_threshold' key
# is not SuperPoint's 'keypoint_threshold': the reference detector ignores it and keeps its
# default 0.005, and so does this one (SuperPoint merges unknown keys without reading them).
confs = {
    "superpoint": {
        "output": "feats-spp",
        "model": {"name": "spp_det"},
        "preprocessing": {"grayscale": True, "resize_h": 512, "resize_w": 512},
        "conf": {"descriptor_dim": 256, "nms_radius": 3, "max_keypoints": 4096,
                 "keypoints_threshold": 0.6},
    }
}


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


LAYERS = ("conv1a", "conv1b", "conv2a", "conv2b", "conv3a", "conv3b", "conv4a", "conv4b",
          "convPa", "convPb", "convDa", "convDb")
SHAPES = {"conv1a": (64, 1, 3), "conv1b": (64, 64, 3), "conv2a": (64, 64, 3),
          "conv2b": (64, 64, 3), "conv3a": (128, 64, 3), "conv3b": (128, 128, 3),
          "conv4a": (128, 128, 3), "conv4b": (128, 128, 3), "convPa": (256, 128, 3),
          "convPb": (65, 256, 1), "convDa": (256, 128, 3), "convDb": (256, 256, 1)}


class SuperPoint:
    """superpoint.py:119-243 on the GPU.  Not an ``nn.Module`` (no autograd: the reference
    only runs it under ``torch.no_grad``), but ``state_dict`` / ``load_state_dict`` / ``eval``
    / ``to`` / ``cuda`` behave as the module's do for inference."""

    default_config = {
        "descriptor_dim": 256,
        "nms_radius": 4,
        "keypoint_threshold": 0.005,
        "max_keypoints": -1,
        "remove_borders": 4,
    }

    def __init__(self, config=None):
        self.config = {**self.default_config, **(config or {})}
        if self.config["descriptor_dim"] != 256:
            raise ValueError("descriptor_dim must be 256 (the descriptor head is fixed)")
        mk = self.config["max_keypoints"]
        if mk == 0 or mk < -1:
            raise ValueError('"max_keypoints" must be positive or "-1"')
        gen = torch.Generator().manual_seed(0)
        self._params = {}
        for name in LAYERS:   # nn.Conv2d's default init (kaiming-uniform a=sqrt(5))
            cout, cin, k = SHAPES[name]
            bound = 1.0 / np.sqrt(cin * k * k)
            self._params[f"{name}.weight"] = (torch.rand(cout, cin, k, k, generator=gen) * 2 - 1) * bound
            self._params[f"{name}.bias"] = (torch.rand(cout, generator=gen) * 2 - 1) * bound
        self.device = torch.device("cpu")
        self._packed = None
        self._ws = {}

    # ------------------------------------------------------------------ parameters
    def state_dict(self):
        return dict(self._params)

    def load_state_dict(self, sd, strict: bool = True):
        """Strict by default, as ``load_network`` calls it (model_io.py:84-88)."""
        missing = [k for k in self._params if k not in sd]
        unexpected = [k for k in sd if k not in self._params]
        if strict and (missing or unexpected):
            raise RuntimeError(f"SuperPoint.load_state_dict: missing {missing}, unexpected {unexpected}")
        for k in self._params:
            if k in sd:
                v = torch.as_tensor(sd[k]).detach().to("cpu", torch.float32)
                if tuple(v.shape) != tuple(self._params[k].shape):
                    raise RuntimeError(f"{k}: shape {tuple(v.shape)} != {tuple(self._params[k].shape)}")
                self._params[k] = v.contiguous()
        self._packed = None
        return self

    def load_network(self, path: str):
        """model_io.load_network for one file: ``torch.load(weights_only=True)``, optional
        'net' wrapper."""
        sd = torch.load(path, map_location="cpu", weights_only=True)
        return self.load_state_dict(sd.get("net", sd))

    def eval(self):
        return self

    def to(self, device):
        self.device = torch.device(device)
        self._packed = None
        self._ws = {}
        return self

    def cuda(self, device=None):
        return self.to("cuda" if device is None else f"cuda:{device}" if isinstance(device, int) else device)

    def packed_weights(self):
        if self._packed is None:
            lib = _lib.load()
            host = [self._params[f"{n}.{t}"].contiguous() for n in LAYERS for t in ("weight", "bias")]
            arr = (_lib.c_void_p * len(host))(*[h.data_ptr() for h in host])
            buf = np.empty(lib.onepose_superpoint_packed_bytes() // 4, dtype=np.float32)
            _lib.check(lib.onepose_superpoint_pack(arr, len(host), buf.ctypes.data), "superpoint_pack")
            self._packed = torch.from_numpy(buf).to(self.device)
        return self._packed

    # ------------------------------------------------------------------ forward
    def capacity(self, h: int, w: int) -> int:
        mk = self.config["max_keypoints"]
        return h * w if mk < 0 else mk

    def _workspace(self, b, h, w):
        key = (b, h, w)
        if key not in self._ws:
            n = _lib.load().onepose_superpoint_workspace_bytes(b, h, w)
            self._ws = {key: torch.empty(n, dtype=torch.uint8, device=self.device)}
        return self._ws[key]

    def detect_raw(self, image, score_map: bool = False, dense: bool = False):
        """image [B,1,H,W] (or [B,H,W]) float on the GPU -> dict of device tensors:
        keypoints [B,K,2] (x, y), scores [B,K], descriptors [B,256,K], counts [B] int32 (K =
        max_keypoints, or H*W for -1; entries past counts[b] are zero); optionally score_map
        [B,H,W] (softmax + pixel shuffle, before NMS) and dense [B,H/8,W/8,256]."""
        if image.device.type != "cuda":
            raise RuntimeError("onepose_amd.SuperPoint runs on a ROCm GPU only")
        if image.dim() == 4:
            if image.shape[1] != 1:
                raise ValueError("SuperPoint takes grayscale images [B,1,H,W]")
            image = image[:, 0]
        img = image.float().contiguous()
        b, h, w = img.shape
        if h % 8 or w % 8:
            raise ValueError(f"image {h}x{w}: sides must be multiples of 8")
        lib = _lib.load()
        k = self.capacity(h, w)
        dev = img.device
        out = {"keypoints": torch.empty(b, k, 2, device=dev),
               "scores": torch.empty(b, k, device=dev),
               "descriptors": torch.empty(b, 256, k, device=dev),
               "counts": torch.empty(b, dtype=torch.int32, device=dev)}
        if score_map:
            out["score_map"] = torch.empty(b, h, w, device=dev)
        if dense:
            out["dense"] = torch.empty(b, h // 8, w // 8, 256, device=dev)
        ws = self._workspace(b, h, w)
        c = self.config
        _lib.check(lib.onepose_superpoint(
            self.packed_weights().data_ptr(), img.data_ptr(), b, h, w, int(c["nms_radius"]),
            float(c["keypoint_threshold"]), int(c["remove_borders"]), k,
            int(reference_align_corners()), out["keypoints"].data_ptr(), out["scores"].data_ptr(),
            out["descriptors"].data_ptr(), out["counts"].data_ptr(), _lib.ptr(out.get("score_map")),
            _lib.ptr(out.get("dense")), ws.data_ptr(), ws.numel(), _lib.stream_ptr(dev)),
            "superpoint")
        return out

    def forward(self, inp):
        """superpoint.py:170-243: per image, keypoints [n,2] (x,y), scores [n],
        descriptors [256,n]."""
        raw = self.detect_raw(inp)
        counts = raw["counts"].cpu().tolist()
        return {"keypoints": [raw["keypoints"][i, :n] for i, n in enumerate(counts)],
                "scores": [raw["scores"][i, :n] for i, n in enumerate(counts)],
                "descriptors": [raw["descriptors"][i, :, :n] for i, n in enumerate(counts)]}

    __call__ = forward


def detect_from_maps(score_map, dense_nhwc, nms_radius=4, keypoint_threshold=0.005,
                     remove_borders=4, max_keypoints=-1, align_corners=None):
    """The detector's tail alone (simple_nms, threshold, remove_borders, top_k, flip,
    sample_descriptors; superpoint.py:47-113, 181-243) from a score map [B,H,W] and a
    normalised dense descriptor map [B,H/8,W/8,256] on the GPU.  Returns detect_raw's dict."""
    if score_map.device.type != "cuda":
        raise RuntimeError("onepose_amd.superpoint runs on a ROCm GPU only")
    if align_corners is None:
        align_corners = reference_align_corners()
    lib = _lib.load()
    s = score_map.float().contiguous()
    d = dense_nhwc.float().contiguous()
    b, h, w = s.shape
    if tuple(d.shape) != (b, h // 8, w // 8, 256):
        raise ValueError(f"dense map {tuple(d.shape)} does not match score map {tuple(s.shape)}")
    k = h * w if max_keypoints < 0 else max_keypoints
    dev = s.device
    out = {"keypoints": torch.empty(b, k, 2, device=dev), "scores": torch.empty(b, k, device=dev),
           "descriptors": torch.empty(b, 256, k, device=dev),
           "counts": torch.empty(b, dtype=torch.int32, device=dev)}
    nws = lib.onepose_superpoint_detect_workspace_bytes(b, h, w)
    ws = torch.empty(nws, dtype=torch.uint8, device=dev)
    _lib.check(lib.onepose_superpoint_detect(
        s.data_ptr(), d.data_ptr(), b, h, w, int(nms_radius), float(keypoint_threshold),
        int(remove_borders), k, int(bool(align_corners)), out["keypoints"].data_ptr(),
        out["scores"].data_ptr(), out["descriptors"].data_ptr(), out["counts"].data_ptr(),
        ws.data_ptr(), nws, _lib.stream_ptr(dev)), "superpoint_detect")
    return out
