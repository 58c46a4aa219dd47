"""Per-object frame pipeline: the whole per-frame hot path of ``inference.py:132-160`` on the
device, with no host round trip and no per-frame re-upload of the object's 3D tensors.

    [SuperPoint (onepose_superpoint)] -> matcher (onepose_match) -> correspondence selection
    -> RANSAC-EPnP -> cm/deg error

The object's descriptors / leaves / 3D points are uploaded once (``inference.py:89-90``
re-uploads them every frame).  With ``object_cache`` (default) the object-only prefix of the
forward -- GAT 0 and the 3D half of self-attention 1 -- is also run once
(``onepose_object_prepare``); each frame's matcher (``onepose_match_cached``) starts from that
state and returns the same bits as the uncached forward (SURVEY.md §8b / §8d F_dep).
All buffers are allocated at construction, so the enqueue
methods only launch kernels on the current stream and can be captured in a HIP graph.

The matcher's ``conf_matrix`` is not kept by default (``with_conf=False``): the reference
driver discards it (``pred, _ = matching_model(inp)``, ``inference.py:146``), and without a
caller buffer the dual-softmax kernel computes the row / column winners from the score matrix
without storing the [B, n1, n3] product (16.8 MB per frame at config 2).

Streaming (``run_stream``): the pose stage of frame k needs one CU (one workgroup per
frame) while the matcher of frame k+1 needs the whole chip, so the two run on separate HIP
streams with two buffer slots; events order matcher(k) -> pose(k) and pose(k) -> the
matcher that next overwrites slot k % 2.  Every frame still runs every kernel.  Staged
(``run_stream(staged=True)``, bench.py's default with a frame bank or a detector): the match
streams run only the GNN layers; the pose stream of frame k runs its final projection, score
GEMM and dual-softmax winners, its pose stage and then the input stage ([detector ->]
transpose [-> self-attention 1]) of the frame that next uses the slot
(``onepose_match_cached_stages``; see ``prime_inputs``).

With a ``detector`` (``onepose_amd.superpoint.SuperPoint``) the pipeline starts from images
(``extract_features.py`` + ``inference.py:143``): each slot owns an image buffer and the
detector writes its keypoints / descriptors straight into that slot's matcher inputs
([B, n1, 2] and [B, 256, n1], n1 = max_keypoints).  The matcher then runs at n1 keypoints, so
the graph-replayed path is exact when the detector fills its top-k (``det_counts`` == n1, the
512x512 crops' usual case); frames with fewer keypoints belong on ``inference.run_frames``,
which runs each frame at its own size.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .matcher import GATsSuperGlue


class _Slot:
    def __init__(self, B, n1, n3, dev, with_conf, lib, L, iters, image_hw=None, precision=0):
        f32 = dict(dtype=torch.float32, device=dev)
        if image_hw is not None:   # detector inputs / outputs (the matcher reads the latter)
            h, w = image_hw
            self.image = torch.zeros(B, h, w, **f32)
            self.kpts2d = torch.zeros(B, n1, 2, **f32)
            self.desc2d = torch.zeros(B, 256, n1, **f32)
            self.det_scores = torch.empty(B, n1, **f32)
            self.det_counts = torch.empty(B, dtype=torch.int32, device=dev)
            self.ws_det_bytes = lib.onepose_superpoint_workspace_bytes(B, h, w)
            self.ws_det = torch.empty(self.ws_det_bytes, dtype=torch.uint8, device=dev)
        self.matches0 = torch.empty(B, n1, dtype=torch.int64, device=dev)
        self.matches1 = torch.empty(B, n3, dtype=torch.int64, device=dev)
        self.mscores0 = torch.empty(B, n1, **f32)
        self.mscores1 = torch.empty(B, n3, **f32)
        self._conf = torch.empty(B, n1, n3, **f32) if with_conf else None
        self.pts2d = torch.empty(B, n1, 2, **f32)
        self.pts3d = torch.empty(B, n1, 3, **f32)
        self.counts = torch.empty(B, dtype=torch.int32, device=dev)
        self.pose = torch.empty(B, 3, 4, dtype=torch.float64, device=dev)
        self.inlier_mask = torch.empty(B, n1, dtype=torch.uint8, device=dev)
        self.n_inliers = torch.empty(B, dtype=torch.int32, device=dev)
        self.status = torch.empty(B, dtype=torch.int32, device=dev)
        self.R_err = torch.empty(B, dtype=torch.float64, device=dev)
        self.t_err = torch.empty(B, dtype=torch.float64, device=dev)
        self.cmd = torch.empty(B, 3, dtype=torch.uint8, device=dev)
        self.ws_match_bytes = _lib.workspace_bytes(lib, B, n1, n3, L, with_conf, precision)
        self.ws_match = torch.empty(self.ws_match_bytes, dtype=torch.uint8, device=dev)
        self.ws_pnp_bytes = lib.onepose_pnp_workspace_bytes(B, n1, iters)
        self.ws_pnp = torch.empty(self.ws_pnp_bytes, dtype=torch.uint8, device=dev)


    @property
    def conf(self):
        """The frame's conf_matrix [B, n1, n3] (only with FramePipeline(with_conf=True); the
        default since round 4 is False, as the reference driver discards it)."""
        if self._conf is None:
            raise RuntimeError("conf_matrix is not kept: build FramePipeline(with_conf=True) to "
                               "read it (the default, like the reference driver, discards it)")
        return self._conf


class FramePipeline:
    def __init__(self, matcher: GATsSuperGlue, keypoints3d, desc3d, leaves, batch: int, n1: int,
                 device, scale: float = 1000.0, reprojection_error: float = 5.0,
                 iterations_count: int = 10000, confidence: float = 0.99, with_conf=False,
                 slots: int = 2, detector=None, image_hw=(512, 512), object_cache: bool = True,
                 gat_tables: bool = True, desc_dtype: str = "fp32"):
        """desc_dtype "fp16": the object's descriptors / leaves and the query descriptors are held
        in fp16 on the device (BASELINE config 5's "fp16 desc"); the kernels convert them as they
        load them, which is the reference's .float() upcast (GATs_SuperGlue.py:219-221), so the
        results are those of the fp32 pipeline on the fp16-rounded inputs, bit for bit."""
        self.lib = _lib.load()
        self.device = torch.device(device)
        self.B, self.n1 = int(batch), int(n1)
        self.scale, self.reproj = float(scale), float(reprojection_error)
        self.iters, self.conf_level = int(iterations_count), float(confidence)
        hp = matcher.hparams
        self.precision = matcher.precision
        self.scale_factor = float(hp["scale_factor"] if isinstance(hp, dict) else hp.scale_factor)
        self.threshold = float(hp["match_threshold"] if isinstance(hp, dict) else hp.match_threshold)
        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        if desc_dtype not in ("fp32", "fp16"):
            raise ValueError(f"desc_dtype {desc_dtype!r}")
        self.desc_dt = _lib.DT_F16 if desc_dtype == "fp16" else _lib.DT_F32
        fdesc = dict(dtype=torch.float16 if desc_dtype == "fp16" else torch.float32, device=dev)
        if desc_dtype == "fp16" and (not object_cache or detector is not None):
            raise ValueError("fp16 descriptors: the object-cached pipeline without a detector")
        self.weights = matcher.packed_weights(dev)
        self.kp3 = torch.as_tensor(np.asarray(keypoints3d), **f32).reshape(-1, 3).contiguous()
        def as_desc(x):
            x = x if torch.is_tensor(x) else torch.as_tensor(np.asarray(x))
            return x.to(**fdesc).reshape(256, -1).contiguous()
        self.desc3d = as_desc(desc3d)
        self.n3 = self.desc3d.shape[1]
        self.leaves = as_desc(leaves)
        self.L = self.leaves.shape[1] // self.n3
        assert self.L * self.n3 == self.leaves.shape[1] and self.kp3.shape[0] == self.n3
        # the object's leaves, transposed once to the point-major layout the GAT layers read
        self.leaves_pm = torch.empty(self.n3 * self.L * 256, **f32)
        _lib.check(self.lib.onepose_prepare_leaves_dt(
            self.leaves.data_ptr(), self.desc_dt, 0, 1, self.n3, self.L, self.leaves_pm.data_ptr(),
            _lib.stream_ptr(dev)), "prepare_leaves")
        # the object-only prefix of the forward (GAT 0 + the 3D half of self-attention 1) and,
        # with gat_tables, the GAT prefix tables, computed once: every frame starts from it
        # (onepose_match_cached; bit-identical to the uncached forward without the tables,
        # equal within rounding with them)
        self.object_cache = None
        self.object_flags = _lib.OBJ_GAT_TABLES if gat_tables else 0
        if object_cache:
            nbytes = _lib.object_cache_bytes(self.lib, self.n3, self.L, self.object_flags,
                                             self.precision)
            self.object_cache = torch.empty(nbytes // 4, **f32)
            wsb = self.lib.onepose_object_prepare_workspace_bytes(self.n3, self.L)
            ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
            _lib.check(self.lib.onepose_object_prepare_dt(
                self.weights.data_ptr(), self.desc3d.data_ptr(), self.desc_dt,
                self.leaves_pm.data_ptr(),
                self.n3, self.L, self.precision, self.object_flags, self.object_cache.data_ptr(),
                ws.data_ptr(), wsb,
                _lib.stream_ptr(dev)), "object_prepare")
            torch.cuda.current_stream(dev).synchronize()
            del ws
        B = self.B
        # per-frame inputs (filled by the caller)
        self.desc2d = torch.zeros(B, 256, n1, **fdesc)
        self.kpts2d = torch.zeros(B, n1, 2, **f32)
        self.K = torch.zeros(B, 3, 3, dtype=torch.float64, device=dev)
        self.pose_gt = torch.zeros(B, 3, 4, dtype=torch.float64, device=dev)
        self.detector = detector
        if detector is not None:
            cap = detector.capacity(*image_hw)
            if cap != n1:
                raise ValueError(f"detector max_keypoints {cap} != pipeline n1 {n1}")
            self.det_weights = detector.to(dev).packed_weights()
        self.image_hw = tuple(image_hw) if detector is not None else None
        self.slots = [_Slot(B, n1, self.n3, dev, with_conf, self.lib, self.L, self.iters,
                            self.image_hw, self.precision) for _ in range(max(1, slots))]

    def __del__(self):
        # drop the library's record of this object cache before its memory goes back to the
        # allocator (onepose_object_release; a later cache at the address is prepared anew)
        cache = self.__dict__.get("object_cache")
        if cache is not None:
            try:
                self.lib.onepose_object_release(cache.data_ptr())
            except Exception:
                pass

    def __getattr__(self, name):
        # slot-0 outputs as attributes (pipe.pose, pipe.matches0, ...) for the common case
        slots = self.__dict__.get("slots")
        if slots is not None and hasattr(slots[0], name):
            return getattr(slots[0], name)
        raise AttributeError(name)

    def set_frames(self, desc2d, kpts2d, K, pose_gt):
        """Copy B frames' inputs into the static buffers (host or device arrays)."""
        self.desc2d.copy_(torch.as_tensor(np.asarray(desc2d)).to(self.desc2d.dtype))
        self.kpts2d.copy_(torch.as_tensor(np.asarray(kpts2d), dtype=torch.float32))
        self.K.copy_(torch.as_tensor(np.asarray(K), dtype=torch.float64).expand_as(self.K))
        self.pose_gt.copy_(torch.as_tensor(np.asarray(pose_gt), dtype=torch.float64)[..., :3, :]
                           .expand_as(self.pose_gt))

    def set_frame_bank(self, desc2d, kpts2d, K, pose_gt):
        """A bank of F steps' inputs ([F, B, ...]: F * B distinct frames) made resident once;
        step k of ``run_stream`` then reads bank entry k % F (F must be a multiple of the slot
        count: entry j always runs in slot j % slots, so its captured graphs stay bound to one
        slot's buffers).  Each entry also gets its own result rows (pose, errors, cm/deg flags,
        inliers, status: ``bank_results``), written by the pose stage of the entry's last run."""
        F = int(np.asarray(desc2d).shape[0]) if not torch.is_tensor(desc2d) else desc2d.shape[0]
        if F % len(self.slots) != 0:
            raise ValueError(f"frame bank of {F} steps is not a multiple of {len(self.slots)} slots")
        dev, B = self.device, self.B

        def dev_t(x, dt, shape):
            return torch.as_tensor(np.asarray(x) if not torch.is_tensor(x) else x,
                                   dtype=dt).reshape(shape).to(dev).contiguous()
        f64 = torch.float64
        self.bank = {"desc2d": dev_t(desc2d, self.desc2d.dtype, (F, B, 256, self.n1)),
                     "kpts2d": dev_t(kpts2d, torch.float32, (F, B, self.n1, 2)),
                     "K": dev_t(K, f64, (F, B, 3, 3)),
                     "pose_gt": dev_t(np.asarray(pose_gt)[..., :3, :] if not torch.is_tensor(pose_gt)
                                      else pose_gt[..., :3, :], f64, (F, B, 3, 4))}
        self.bank_results = {"pose": torch.zeros(F, B, 3, 4, dtype=f64, device=dev),
                             "R_err": torch.zeros(F, B, dtype=f64, device=dev),
                             "t_err": torch.zeros(F, B, dtype=f64, device=dev),
                             "cmd": torch.zeros(F, B, 3, dtype=torch.uint8, device=dev),
                             "n_inliers": torch.zeros(F, B, dtype=torch.int32, device=dev),
                             "status": torch.full((F, B), -1, dtype=torch.int32, device=dev)}

    @property
    def bank_size(self) -> int:
        return self.bank["desc2d"].shape[0] if getattr(self, "bank", None) is not None else 0

    def set_images(self, images, slot=None):
        """Copy B images ([B, H, W] or [B, 1, H, W], float in [0, 1]) into one slot's image
        buffer, or into every slot when slot is None."""
        img = torch.as_tensor(np.asarray(images) if not torch.is_tensor(images) else images,
                              dtype=torch.float32).reshape(self.B, *self.image_hw)
        for o in (self.slots if slot is None else [self.slots[slot]]):
            o.image.copy_(img)

    def _inputs(self, o, frame=None):
        if self.detector is not None:
            return o.desc2d, o.kpts2d
        if frame is not None:
            return self.bank["desc2d"][frame], self.bank["kpts2d"][frame]
        return self.desc2d, self.kpts2d

    def enqueue_detect(self, slot: int = 0):
        """SuperPoint on the slot's images into the slot's matcher inputs."""
        o = self.slots[slot]
        c = self.detector.config
        h, w = self.image_hw
        from .superpoint import reference_align_corners
        _lib.check(self.lib.onepose_superpoint(
            self.det_weights.data_ptr(), o.image.data_ptr(), self.B, h, w, int(c["nms_radius"]),
            float(c["keypoint_threshold"]), int(c["remove_borders"]), self.n1,
            int(reference_align_corners()), o.kpts2d.data_ptr(), o.det_scores.data_ptr(),
            o.desc2d.data_ptr(), o.det_counts.data_ptr(), 0, 0, o.ws_det.data_ptr(),
            o.ws_det_bytes, _lib.stream_ptr(self.device)), "onepose_superpoint")

    def enqueue_front(self, slot: int = 0, frame=None):
        """The stage that runs on a match stream: [detector ->] matcher (on frame-bank entry
        `frame` when given)."""
        if self.detector is not None:
            self.enqueue_detect(slot)
        self.enqueue_match(slot, frame)

    def enqueue_match(self, slot: int = 0, frame=None, stages=None):
        """The matcher on the slot (frame-bank entry `frame` when given).  `stages`
        (first, last) runs that range of the forward's stages (onepose_match_cached_stages):
        STAGE_INPUTS (the frame's descriptors into the slot's workspace, its counters zeroed,
        the object cache's header checked), STAGE_LAYER0 + i (GNN layer i), STAGE_FINAL (final
        projection), STAGE_SCORE (score GEMM), STAGE_WINNERS (dual softmax winners + mutual
        check) -- each on what the stages before left in the workspace; None: the whole
        forward."""
        o = self.slots[slot]
        s = _lib.stream_ptr(self.device)
        desc2d, _ = self._inputs(o, frame)
        if stages is not None and self.object_cache is None:
            raise ValueError("the matcher runs by stages only with the object cache")
        if stages is None:
            self._primed = False   # the slot's staged input (if any) is overwritten
            stages = (_lib.STAGE_INPUTS, _lib.STAGE_WINNERS)
        if self.object_cache is not None:
            _lib.check(self.lib.onepose_match_cached_stages(
                self.weights.data_ptr(), desc2d.data_ptr(), self.desc_dt, 256 * self.n1,
                self.object_cache.data_ptr(), self.leaves_pm.data_ptr(), 0,
                self.B, self.n1, self.n3, self.L, self.scale_factor, self.threshold,
                self.precision, self.object_flags, o.matches0.data_ptr(), o.matches1.data_ptr(),
                o.mscores0.data_ptr(), o.mscores1.data_ptr(), _lib.ptr(o._conf),
                o.ws_match.data_ptr(), o.ws_match_bytes, stages[0], stages[1], s),
                "onepose_match_cached")
            return
        _lib.check(self.lib.onepose_match_prepared_ex(
            self.weights.data_ptr(), desc2d.data_ptr(), 256 * self.n1,
            self.desc3d.data_ptr(), 0, self.leaves_pm.data_ptr(), 0,
            self.B, self.n1, self.n3, self.L, self.scale_factor, self.threshold, self.precision,
            o.matches0.data_ptr(), o.matches1.data_ptr(), o.mscores0.data_ptr(),
            o.mscores1.data_ptr(), _lib.ptr(o._conf), o.ws_match.data_ptr(),
            o.ws_match_bytes, s), "onepose_match_prepared")

    fused_pose = True   # enqueue_pose's default: onepose_pose_stage (two launches)

    def enqueue_pose(self, slot: int = 0, fused: bool | None = None, frame=None):
        """Selection -> RANSAC-EPnP -> cm/deg errors for the slot's frames: two launches
        (onepose_pose_stage), or the three separate entry points (fused=False).  With `frame`
        (a frame-bank entry) the entry's K and ground truth are read and its result rows
        written (``bank_results``)."""
        fused = self.fused_pose if fused is None else fused
        o = self.slots[slot]
        s = _lib.stream_ptr(self.device)
        lib = self.lib
        _, kpts2d = self._inputs(o, frame)
        if frame is not None:
            K, pose_gt = self.bank["K"][frame], self.bank["pose_gt"][frame]
            r = {k: v[frame] for k, v in self.bank_results.items()}
        else:
            K, pose_gt = self.K, self.pose_gt
            r = {"pose": o.pose, "R_err": o.R_err, "t_err": o.t_err, "cmd": o.cmd,
                 "n_inliers": o.n_inliers, "status": o.status}
        if fused:
            _lib.check(lib.onepose_pose_stage(
                o.matches0.data_ptr(), kpts2d.data_ptr(), self.n1 * 2, self.kp3.data_ptr(), 0,
                self.B, self.n1, self.n3, self.scale, K.data_ptr(), 9, self.reproj,
                self.iters, self.conf_level, pose_gt.data_ptr(), 12, o.pts2d.data_ptr(),
                o.pts3d.data_ptr(), o.counts.data_ptr(), r["pose"].data_ptr(),
                o.inlier_mask.data_ptr(), r["n_inliers"].data_ptr(), r["status"].data_ptr(),
                r["R_err"].data_ptr(), r["t_err"].data_ptr(), r["cmd"].data_ptr(),
                o.ws_pnp.data_ptr(), o.ws_pnp_bytes, s), "pose_stage")
            return
        if frame is not None:
            raise ValueError("frame-bank entries run the fused pose stage")
        _lib.check(lib.onepose_select_correspondences(
            o.matches0.data_ptr(), kpts2d.data_ptr(), self.n1 * 2, self.kp3.data_ptr(), 0,
            self.B, self.n1, self.n3, self.scale, o.pts2d.data_ptr(), o.pts3d.data_ptr(),
            o.counts.data_ptr(), s), "select_correspondences")
        _lib.check(lib.onepose_pnp_ransac(
            o.pts2d.data_ptr(), o.pts3d.data_ptr(), o.counts.data_ptr(), self.n1,
            self.K.data_ptr(), 9, self.B, self.scale, self.reproj, self.iters, self.conf_level,
            o.pose.data_ptr(), o.inlier_mask.data_ptr(), o.n_inliers.data_ptr(),
            o.status.data_ptr(), o.ws_pnp.data_ptr(), o.ws_pnp_bytes, s), "pnp_ransac")
        _lib.check(lib.onepose_pose_errors(
            o.pose.data_ptr(), self.pose_gt.data_ptr(), 12, self.B, o.R_err.data_ptr(),
            o.t_err.data_ptr(), o.cmd.data_ptr(), s), "pose_errors")

    def enqueue(self, slot: int = 0):
        self.enqueue_front(slot)
        self.enqueue_pose(slot)

    def capture(self, slot: int = 0, pool=None) -> "torch.cuda.CUDAGraph":
        """Capture one whole step (``enqueue(slot)``: ~60 launches) as a HIP graph.

        Every launch reads and writes this pipeline's static buffers, so replaying the graph
        after ``set_frames`` (or after writing new frames into ``desc2d``/``kpts2d``/``K``/
        ``pose_gt`` in place) runs the full hot path for the new inputs; the graph removes the
        per-launch host overhead, not any work."""
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=pool):
            self.enqueue(slot)
        return g

    # ---- staged stages: the forward's short stages on the pose streams ----
    # With a frame bank and the object cache, step g runs bank entry g % F in slot g % n.  The
    # match stream runs the GNN layers from ``staged_head`` up to ``staged_split``; the pose
    # stream runs the rest of the step's forward (default: the final projection, the score GEMM,
    # the dual-softmax winners + mutual check), its pose stage, and then the input stage -- with
    # the stages before ``staged_head`` -- of step g + n, the next step to use the slot.  These
    # short stages thus run beside the other streams' layers instead of on this stream's launch
    # chain.  Every step still runs all of its forward and its pose stage; the step counter
    # carries over between run_stream calls so that the staged inputs are the ones the next
    # call's first steps need.  prime_inputs() stages the first n steps.
    _primed = False
    _next_step = 0
    staged_split = _lib.STAGE_FINAL   # first stage of the forward on the pose stream

    # first stage of the forward on the match streams: the stages before it run ahead, with the
    # input stage, at the end of the slot's previous pose stage (LAYER0: the input stage alone)
    staged_head = _lib.STAGE_LAYER0

    def _staged_split(self):
        k, h = self.staged_split, self.staged_head
        if not _lib.STAGE_LAYER0 <= h < k <= _lib.STAGE_WINNERS:
            raise ValueError(f"staged_head {h} / staged_split {k}")
        return (h, k - 1), (k, _lib.STAGE_WINNERS)

    def staged_ok(self) -> bool:
        """Staged runs need the object cache and inputs known ahead: a frame bank, or the
        detector's per-slot images (each step re-detects its slot's image)."""
        return self.object_cache is not None and (self.detector is not None
                                                  or self.bank_size > 0)

    def enqueue_inputs(self, slot: int, frame):
        """The matcher's input stage for bank entry `frame` (None: the slot's detector
        outputs, after running the detector on the slot's image) into `slot`, with the stages
        before ``staged_head``."""
        if self.detector is not None:
            self.enqueue_detect(slot)
        self.enqueue_match(slot, frame, stages=(_lib.STAGE_INPUTS, self.staged_head - 1))

    def prime_inputs(self):
        """Stage the inputs of the next len(slots) steps on the current stream (before the first
        staged ``run_stream``, and again after anything else used the slots' workspaces)."""
        if not self.staged_ok():
            raise ValueError("staged inputs need the object cache and a frame bank or a detector")
        n, F = len(self.slots), self.bank_size
        for g in range(self._next_step, self._next_step + n):
            self.enqueue_inputs(g % n, g % F if F else None)
        self._primed = True

    def capture_stages(self, pool=None, staged: bool = False):
        """Capture, per buffer slot, the front stage ([detector ->] matcher) and the pose stage
        as two HIP graphs (for ``run_stream(graphs=...)``).  With a frame bank, one pair per
        bank entry j instead (slot j % slots, the entry's inputs and result rows).  `staged`:
        the matcher graph is the GNN layers before ``staged_split``, the pose graph the rest of
        the forward, the pose stage and the input stage of entry (j + slots) % F (for
        ``run_stream(staged=True)``)."""
        out = []
        F, n = self.bank_size, len(self.slots)
        if staged and not self.staged_ok():
            raise ValueError("staged inputs need the object cache and a frame bank or a detector")
        head, tail = self._staged_split()
        for j in range(F or n):
            sl, fr = j % n, (j if F else None)
            gm, gp = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(gm, pool=pool):
                if staged:
                    self.enqueue_match(sl, fr, stages=head)
                else:
                    self.enqueue_front(sl, fr)
            with torch.cuda.graph(gp, pool=pool):
                if staged:
                    self.enqueue_match(sl, fr, stages=tail)
                self.enqueue_pose(sl, frame=fr)
                if staged:
                    self.enqueue_inputs(sl, (j + n) % F if F else None)
            out.append((gm, gp))
        self._primed = False   # (the non-staged captures above mark it too)
        self._captured_split = (head, tail) if staged else None
        return out

    def run_stream(self, steps: int, match_stream=None, pose_stream=None, graphs=None,
                   marks=None, match_streams: int = 1, pose: bool = True,
                   pose_streams: int = 1, staged: bool = False):
        """Enqueue `steps` frames (batches) with matcher(k+1) overlapping pose(k); with
        `graphs` (from ``capture_stages``) each stage is one graph replay.  With
        `match_streams` = m > 1, consecutive frames' matchers run on m streams concurrently
        (frame k on stream k % m; needs >= m + 1 buffer slots), filling the CUs that one
        frame's kernels leave idle.  Every frame still runs every kernel.  All streams are
        joined into the first match stream at the end; the caller synchronises.  With
        `pose_streams` = p > 1, frame k's pose stage runs on pose stream k % p (each stage reads
        and writes only its slot's buffers), so two frames' pose stages that become ready
        together -- the last frames of a batch -- run side by side instead of one after the
        other.  `marks` (a list) receives per step (start, matcher done, pose done) timing
        events.  With a frame bank (``set_frame_bank``), step k runs bank entry k % F; `graphs`
        then holds one pair per entry (``capture_stages``).  `staged` (graphs from
        ``capture_stages(staged=True)``, after ``prime_inputs``): the steps continue the bank
        from the previous staged call, the match streams run the GNN layers before
        ``staged_split``, and each pose stream runs the rest of the step's forward before its
        pose stage and the inputs of the step that next uses the slot after it (see
        ``prime_inputs``)."""
        ms0 = match_stream or torch.cuda.current_stream(self.device)
        F = self.bank_size
        g0 = 0
        if not staged:
            self._primed = False   # whole forwards (graphs or not) overwrite the staged inputs
        if staged:
            if not self.staged_ok():
                raise ValueError("staged inputs need the object cache and a frame bank or a "
                                 "detector")
            if not self._primed:
                raise RuntimeError("run_stream(staged=True): call prime_inputs() first")
            if not pose:
                raise ValueError("staged inputs are staged by the pose stages")
            g0 = self._next_step
            head, tail = self._staged_split()
            if graphs and getattr(self, "_captured_split", None) != (head, tail):
                raise ValueError("graphs were not captured with capture_stages(staged=True) "
                                 "for this staged_split")
        ps = pose_stream or getattr(self, "_pose_stream", None)
        if ps is None:
            ps = self._pose_stream = torch.cuda.Stream(
                self.device, priority=getattr(self, "pose_priority", 0))
        pextra = getattr(self, "_pose_streams", [])
        while len(pextra) < pose_streams - 1:
            pextra.append(torch.cuda.Stream(self.device,
                                            priority=getattr(self, "pose_priority", 0)))
        self._pose_streams = pextra
        pss = [ps] + pextra[:max(1, pose_streams) - 1]
        extra = getattr(self, "_match_streams", [])
        while len(extra) < match_streams - 1:
            extra.append(torch.cuda.Stream(self.device,
                                           priority=getattr(self, "match_priority", 0)))
        self._match_streams = extra
        mss = [ms0] + extra[:match_streams - 1]
        n = len(self.slots)
        assert n >= len(mss) + (1 if len(mss) > 1 else 0), "need more buffer slots than streams"
        matched = [torch.cuda.Event() for _ in range(n)]
        posed = [torch.cuda.Event() for _ in range(n)]
        used = [False] * n
        for s in mss[1:]:
            s.wait_stream(ms0)                    # inputs written on the caller's stream
        for k in range(steps):
            g = g0 + k                            # the bank step (k unless staged)
            sl = g % n
            ms = mss[k % len(mss)]
            mk = [torch.cuda.Event(enable_timing=True) for _ in range(3)] if marks is not None \
                else None
            with torch.cuda.stream(ms):
                if used[sl]:                      # slot's previous pose stage has read it
                    ms.wait_event(posed[sl])
                if mk:
                    mk[0].record(ms)
                if graphs:
                    graphs[g % len(graphs)][0].replay()
                elif staged:
                    self.enqueue_match(sl, g % F if F else None, stages=head)
                else:
                    self.enqueue_front(sl, g % F if F else None)
                matched[sl].record(ms)
                if mk:
                    mk[1].record(ms)
            ps = pss[k % len(pss)]
            with torch.cuda.stream(ps):
                ps.wait_event(matched[sl])
                if pose:   # (False: a diagnostic of the matcher streams alone, bench.py)
                    if graphs:
                        graphs[g % len(graphs)][1].replay()
                    else:
                        if staged:
                            self.enqueue_match(sl, g % F if F else None, stages=tail)
                        self.enqueue_pose(sl, frame=g % F if F else None)
                        if staged:
                            self.enqueue_inputs(sl, (g + n) % F if F else None)
                posed[sl].record(ps)
                if mk:
                    mk[2].record(ps)
            used[sl] = True
            if mk:
                marks.append(mk)
        for s in mss[1:]:
            ms0.wait_stream(s)
        for s in pss:
            ms0.wait_stream(s)
        if staged:
            self._next_step = g0 + steps
        return pss[0]
