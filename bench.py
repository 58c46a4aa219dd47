"""Benchmark: query frames/sec of the OnePose GATsSPG hot path on MI355X.

One step = one batch of synthetic query frames (config 2: 1024 keypoints x 4096 3D points,
L = 8 leaves, batch 1 per GPU) pushed through the whole per-frame path of inference.py:
GATsSPG matcher (12 layers, dual softmax, mutual NN; conf_matrix materialised) ->
correspondence selection -> RANSAC-EPnP -> cm/deg error vs GT.  Inputs are resident in HBM
before the timed region; nothing is cached across steps.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N  (one rank/GPU)
    python bench.py --e2e      (extra measurement: each step starts from 512x512 images --
                                SuperPoint on the GPU produces the 1k query keypoints)

Multi-GPU: frames are independent given the object, so each rank runs its own frames
(weak scaling) and the only exchange is one all-gather of per-frame poses and cm/deg flags
at the end of the timed region.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "query frames/sec (1k kpts × 4k 3D pts) + cm/deg pose err, 1/2/4/8 GPU"
FP32_MFMA_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: f32-input MFMA dense peak
BF16_MFMA_PEAK_TFLOPS = 2500.0    # MI355X_MICROARCH.md: "~2.5 PF dense" bf16 MFMA
HBM_PEAK_GBS = 8000.0             # MI355X_MICROARCH.md: HBM3E spec
# kernels that record device stamps (onepose_profile_begin_device): timeable inside graphs
STAMPED = {"qkv_gemm", "mlp1_gemm", "mlp2_gemm", "final_gemm", "score_gemm"}


def superpoint_conv_flops(h, w):
    """Algorithmic FLOPs of SuperPoint's MFMA convolutions for one h x w image
    (superpoint.py:147-162; conv1a, a direct kernel, excluded; convPb at its 65 outputs)."""
    layers = [(1, 64, 64, 3), (2, 64, 64, 3), (2, 64, 64, 3), (4, 64, 128, 3), (4, 128, 128, 3),
              (8, 128, 128, 3), (8, 128, 128, 3), (8, 128, 256, 3), (8, 256, 65, 1),
              (8, 128, 256, 3), (8, 256, 256, 1)]   # (downsampling, cin, cout, k) from conv1b
    return sum(2 * (h // d) * (w // d) * co * ci * k * k for d, ci, co, k in layers)


def cross_cached(cached, B):
    """Whether the cached forward also takes cross-attention 1's frame-independent 3D half
    (the 3D side's q / k / v projections, KV and the x range of its MLP conv 1) from the
    object cache: at every batch since round 2's per-side layer choices (matcher.hip,
    side_tiles); B is kept for the callers' symmetry with frame_flops."""
    del B
    return cached


def frame_flops(n1, n3, L, cached, B=1):
    """algorithmic MFMA FLOPs per frame, F, or F_dep when the object-only
    prefix (GAT 0 + the 3D half of self-attention 1) is cached per object.  With cross-
    attention 1's 3D half cached too (cross_cached), half of that layer's per-3D-token work
    (q, k, v projections 6 C^2, KV 2 C dh, W1a x 4 C^2 = 688,128 FLOP) is not per frame."""
    f = 11141120 * (n1 + n3) + 512 * n1 * n3 + 2048 * (L + 2) * n3
    if not cached:
        return f
    f -= 1376256 * n3 + 512 * (L + 2) * n3
    return f - 688128 * n3 if cross_cached(cached, B) else f


def executed_mfma_flops(n1, n3, cached):
    """MFMA FLOPs the kernels actually execute per frame (as opposed to frame_flops' algorithmic
    count, which prices the reference's merge conv and attention apply that the Mf fold removes):
    per attention layer and token QKV 2*768*256, the KV partials 4 heads x 2*64*64 (QKV
    epilogue), MLP conv 1 2*512*512, MLP conv 2 2*256*512; the cached forward skips the 3D side
    of self-attention 1 and, in cross-attention 1, the 3D side's QKV, KV partials and the
    W1a x half of its MLP conv 1; final projection 2*256*256 per token; score 2*256*n1*n3.
    (The KV fold's Mf = C KV, 16.8 MFLOP per source side and layer, runs on VALU FMAs.)"""
    qkv, kvp, m1, m2 = 2 * 768 * 256, 4 * 2 * 64 * 64, 2 * 512 * 512, 2 * 256 * 512
    full = qkv + kvp + m1 + m2
    f2 = 8 * n1 * full
    f3 = n3 * ((0 + (m1 // 2 + m2) + 6 * full) if cached else 8 * full)
    return f2 + f3 + 2 * 256 * 256 * (n1 + n3) + 2 * 256 * n1 * n3


def kernel_work(kind, B, n1, n3, L, cached=False):
    """Algorithmic work of ONE launch of each matcher kernel kind: (amount, unit, bound).
    GEMM-shaped kernels: FLOPs; byte-moving kernels: bytes that must cross HBM.  With the
    object cache, one of a frame's 8 launches of each attention GEMM has the 2D side only, so
    the figure is the frame's work of that kind / 8 (the average launch)."""
    T = B * (n1 + n3) - (B * n3 / 8 if cached else 0)
    xc = cross_cached(cached, B)   # cross-attention 1: the 3D side's QKV and W1a x cached
    Tq = T - (B * n3 / 8 if xc else 0)
    T1 = T - (B * n3 / 16 if xc else 0)   # half of that layer's 3D MLP-conv-1 K range
    C = 256
    table = {
        "qkv_gemm": (2 * 3 * C * C * Tq, "flop", "mfma"),      # [q | k v] = Wqkv x
        "mlp1_gemm": (2 * 2 * C * 2 * C * T1, "flop", "mfma"),   # [W1a | Mf] [x ; QZ]
        "mlp2_gemm": (2 * 2 * C * C * T, "flop", "mfma"),
        "final_gemm": (2 * C * C * B * (n1 + n3), "flop", "mfma"),   # once per frame, all tokens
        "score_gemm": (2 * C * n1 * n3 * B, "flop", "mfma"),
        # GAT: leaves once + the 3D descriptors in and out (fp32)
        "gat": (4 * C * n3 * B * (L + 2), "byte", "hbm"),
        # conf: read S (fp32); the pipeline keeps no conf_matrix (the reference discards it)
        "conf": (4 * n1 * n3 * B, "byte", "hbm"),
    }
    return table.get(kind)


def pmc_traffic(kernel, subdir="pmc"):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/r*/<subdir>/pmc_traffic.json, written by tools/gpu_r03_b.sh + tools/pmc_summary.py:
    FETCH_SIZE x2 (gfx950) + WRITE_SIZE, separate rocprofv3 passes; "pmc" = config 2 fp32,
    "pmc_c5" = config 5 bf16).  None if absent."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*", subdir, "pmc_traffic.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    k = d.get("kernels", {}).get(kernel)
    if not k or k.get("hbm_bytes") is None:
        return None, None
    return float(k["hbm_bytes"]), os.path.relpath(files[-1], REPO)


def profile_kinds(lib):
    names = []
    k = 0
    while True:
        n = lib.onepose_profile_kind_name(k)
        if n is None:
            break
        names.append(n.decode())
        k += 1
    return names


def run_profiled(lib, pipe, steps, mask, cap):
    from onepose_amd import _lib
    _lib.check(lib.onepose_profile_begin(mask, cap), "profile_begin")
    for _ in range(steps):
        pipe.enqueue()
    kinds = np.zeros(cap, np.int32)
    ms = np.zeros(cap, np.float32)
    cnt = np.zeros(1, np.int32)
    _lib.check(lib.onepose_profile_end(kinds.ctypes.data, ms.ctypes.data, cap, cnt.ctypes.data),
               "profile_end")
    n = int(cnt[0])
    return kinds[:n], ms[:n]


def cpu_baseline(sd, data, frames, obj, seconds=15.0, detector_image=None):
    """The reference's CPU path on the host: the PyTorch-CPU restatement of the matcher
    (oracle/matcher_torch.py, pinned to the reference's fixtures) with every host thread, then
    the C RANSAC-EPnP oracle (OpenCV 4.4's algorithm).  SURVEY §8d: 2 warm-ups, then the median
    of >= 5 calls (bounded to ~`seconds`), matcher and PnP timed separately.  With
    `detector_image` also one SuperPoint oracle pass per frame."""
    import torch
    from oracle import matcher_torch as MT
    from oracle import pnp_oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(threads)
    one = {k: v[:1] for k, v in data.items()}
    tsd = MT.to_torch(sd)
    tm, tp = [], []
    t0 = time.perf_counter()
    for i in range(2 + 15):
        a = time.perf_counter()
        pred, _ = MT.forward(tsd, one)
        b = time.perf_counter()
        p2, p3 = O.select_correspondences(pred["matches0"], one["keypoints2d"][0],
                                          one["keypoints3d"][0], 1000.0)
        O.pnp_ransac(p2, p3, frames[0].K, scale=1000.0)
        c = time.perf_counter()
        if i >= 2:
            tm.append(b - a)
            tp.append(c - b)
        if i >= 6 and time.perf_counter() - t0 > seconds:
            break
    per_frame = float(np.median(tm) + np.median(tp))
    sample = (f"1 frame of the timed workload, 2 warm-ups + median of {len(tm)}: matcher "
              f"{np.median(tm) * 1e3:.1f} ms (PyTorch-CPU restatement of GATsSuperGlue.forward, "
              f"{threads} threads) + RANSAC-EPnP {np.median(tp) * 1e3:.1f} ms (C restatement of "
              f"OpenCV 4.4 solvePnPRansac, 1 thread)")
    if detector_image is not None:
        from onepose_amd import synthetic
        from oracle import superpoint_torch as ST
        ssd = ST.to_torch(synthetic.superpoint_state_dict(0))
        ts = []
        for i in range(2 + 5):
            t1 = time.perf_counter()
            ST.forward(ssd, detector_image, nms_radius=3, keypoint_threshold=0.005,
                       remove_borders=4, max_keypoints=data["keypoints2d"].shape[1])
            if i >= 2:
                ts.append(time.perf_counter() - t1)
        t_sp = float(np.median(ts))
        per_frame += t_sp
        sample += (f"; plus SuperPoint (PyTorch-CPU restatement, {threads} threads) on one "
                   f"{detector_image.shape[0]}x{detector_image.shape[1]} image: "
                   f"{t_sp * 1e3:.1f} ms (median of 5)")
    return {"value": 1.0 / per_frame, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": sample}


def summarize_pose(res, world, B, F, steps):
    """cm/deg and inlier statistics over every timed frame, from the gathered result rows
    (pose 12, R_err, t_err, cmd 1/3/5, inliers, status, global frame id; any row order).

    With a frame bank of F steps (F > 0), row g is global frame g of one sequence: step j's
    global batch is frames [j world B, (j + 1) world B) and step k of the timed region runs bank
    entry k % F, so a row's weight is the number of timed steps that ran its entry.  Without a
    bank (F = 0) the rows are the one batch every step replays, weight 1 each."""
    res = res[np.argsort(res[:, 19], kind="stable")]
    n_rows = world * B * (F or 1)
    assert np.array_equal(res[:, 19], np.arange(n_rows)), "gathered frame order"
    if F:
        entry = (res[:, 19] // (world * B)).astype(np.int64)
        w = np.bincount(np.arange(steps) % F, minlength=F)[entry].astype(np.float64)
        assert w.sum() == world * B * steps
    else:
        w = np.ones(len(res))

    def wmean(x):
        return float((w * x).sum() / w.sum())
    rep = np.repeat(np.arange(len(res)), w.astype(np.int64))
    return {"frames": int(w.sum()), "distinct_frames": int((w > 0).sum()),
            "cmd1": wmean(res[:, 14]), "cmd3": wmean(res[:, 15]), "cmd5": wmean(res[:, 16]),
            "R_err_deg_mean": wmean(res[:, 12]), "t_err_cm_mean": wmean(res[:, 13]),
            "R_err_deg_median": float(np.median(res[rep, 12])),
            "t_err_cm_median": float(np.median(res[rep, 13])),
            "n_inliers_mean": wmean(res[:, 17]),
            "status_ok": wmean((res[:, 18] == 0).astype(np.float64)),
            "source": (f"every timed frame: a bank of {F} steps x {B} frame(s) x {world} rank(s) "
                       f"of distinct synthetic frames, step k runs entry k % {F}") if F
                      else "the last step's frames (one batch replayed every step)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--settle-steps", type=int, default=60,
                    help="at least this many steps of the timed schedule run back to back "
                         "right before the timed region, the W warm-up steps last (the GPU "
                         "reaches its loaded clock within ~40 ms of sustained work: a 20-step "
                         "region after 5 warm-ups reads ~6%% below one after 50, DESIGN.md 4b)")
    ap.add_argument("--batch", type=int, default=1, help="frames per GPU per step")
    ap.add_argument("--n1", type=int, default=1024)
    ap.add_argument("--n3", type=int, default=4096)
    ap.add_argument("--leaf", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--serial", action="store_true",
                    help="one stream: step k+1 starts after step k's pose stage (default: the "
                         "pose stage of step k overlaps the matcher of step k+1 on 2 streams)")
    ap.add_argument("--diag-steps", action="store_true",
                    help="diagnostic: record an event after every timed step and report the "
                         "per-step GPU times")
    ap.add_argument("--match-streams", type=int, default=2,
                    help="consecutive frames' matchers on this many concurrent streams "
                         "(default 2: one frame's kernels leave CUs idle; 1 = one at a time)")
    ap.add_argument("--pose-streams", type=int, default=0,
                    help="pose stages of consecutive steps on this many streams (default: one per "
                         "matcher stream, so the last frames' pose stages run side by side)")
    ap.add_argument("--eager", action="store_true",
                    help="launch every kernel from the host each step instead of replaying "
                         "captured HIP graphs")
    ap.add_argument("--stage-marks", action="store_true",
                    help="diagnostic: per-step timing events in the timed region -> stage_ms "
                         "(they cost ~0.5%% of the frame rate, so they are off by default)")
    ap.add_argument("--no-stamps", action="store_true",
                    help="diagnostic: no device stamps in the timed region (roofline then "
                         "reports the serial profile pass)")
    ap.add_argument("--slots", type=int, default=0,
                    help="frame buffer slots (default: the smallest count >= match streams + 1 "
                         "that divides --frames)")
    ap.add_argument("--frames", type=int, default=64,
                    help="frame bank: this many steps' distinct query frames (x batch x ranks) are "
                         "resident before timing and step k runs bank entry k %% frames; the pose "
                         "summary covers every timed frame (0: one batch of frames replayed)")
    ap.add_argument("--precision", choices=["fp32", "bf16", "fp32_split"], default="fp32",
                    help="matcher attention-layer GEMMs: fp32 MFMA (the reference's numerics, "
                         "default) or bf16 MFMA with fp32 accumulation (BASELINE config 5)")
    ap.add_argument("--desc-dtype", choices=["fp32", "fp16"], default="fp32",
                    help="the object's and the query frames' descriptors as held in HBM (fp16: "
                         "BASELINE config 5's 'fp16 desc'; the kernels convert them as they load "
                         "them, the reference's .float() upcast)")
    ap.add_argument("--no-object-cache", action="store_true",
                    help="run GAT 0 and the 3D half of self-attention 1 every frame instead of "
                         "once per object (onepose_match_prepared_ex instead of _cached)")
    ap.add_argument("--e2e", action="store_true",
                    help="start each step from images: SuperPoint (max_keypoints = n1, nms 3, "
                         "threshold 0.005) on the GPU produces the query keypoints/descriptors")
    ap.add_argument("--image-size", type=int, default=512)
    ap.add_argument("--diag-no-pose", action="store_true",
                    help="diagnostic only (not the metric): skip the pose stage in the timed "
                         "region, to measure what it costs the matcher streams")
    ap.add_argument("--match-priority", type=int, default=0,
                    help="diagnostic: HIP stream priority of the second and later matcher streams "
                         "(lower = higher; the caller's stream keeps the default)")
    ap.add_argument("--pose-priority", type=int, default=0,
                    help="diagnostic: HIP stream priority of the pose stream (lower = higher)")
    ap.add_argument("--unfused-pose", action="store_true",
                    help="pose stage as select + RANSAC-EPnP + errors (4 launches) instead of "
                         "onepose_pose_stage (2)")
    ap.add_argument("--no-staged-inputs", action="store_true",
                    help="run each step's matcher input stage (transpose_in) at the head of its "
                         "matcher instead of at the end of the slot's previous pose stage")
    ap.add_argument("--staged-split", type=int, default=0,
                    help="staged mode: the forward's first stage on the pose stream "
                         "(onepose_match_cached_stages: 1 + i = GNN layer i, 13 = final "
                         "projection, 14 = score GEMM, 15 = dual-softmax winners; 0 = the "
                         "measured best for the precision: 13 for fp32 / fp32_split, 15 for "
                         "bf16, profiles/r06/staged3, profiles/r06/prec)")
    ap.add_argument("--staged-head", type=int, default=0,
                    help="staged mode: the forward's first stage on the match streams; the "
                         "stages before it run with the input stage at the end of the slot's "
                         "previous pose stage (1 = the input stage alone, 3 = with "
                         "self-attention 1's 2D half; 0 = the measured best: 1 for bf16 "
                         "attention at up to 1024 x 4096, else 3, profiles/r06/head)")
    ap.add_argument("--diag-repeats", type=int, default=0,
                    help="diagnostic: after the timed region, time it again this many times "
                         "and report those ms/step too (value always comes from the first)")
    args = ap.parse_args()

    from onepose_amd import distributed as D
    world, rank, local = D.env()
    # ONEPOSE_REHEARSE_ONE_GPU=1: every rank on device 0 over gloo -- rehearses the N>1 code
    # path (sharding, barrier, result gather, max-over-ranks) on a one-GPU box; not a
    # scaling measurement
    rehearse = os.environ.get("ONEPOSE_REHEARSE_ONE_GPU") == "1"
    local = 0 if rehearse else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pg = None
    if D.init("gloo" if rehearse else "nccl", dev):   # one process per GPU over RCCL
        import torch.distributed as dist
        pg = dist

    from onepose_amd import _lib, matcher, synthetic
    from onepose_amd.pipeline import FramePipeline
    lib = _lib.load()

    B, n1, n3, L = args.batch, args.n1, args.n3, args.leaf
    sd = synthetic.make_state_dict(0)
    # One object's batch (BASELINE config 4): every rank builds the same object
    # and weights; the global batch is world * B frames of that object's sequence, generated
    # from one seed, and this rank runs its contiguous frame_shard slice of it.  The gathered
    # result rows come back in global frame order.
    n_global = world * B
    fs, fe = D.frame_shard(n_global, world, rank)
    data, obj, frames = synthetic.make_matcher_inputs(n1, n3, L, seed=0, frame_ids=range(fs, fe))
    F = max(0, args.frames)
    if args.e2e:
        F = 0   # the detector path reads each slot's own images (no query-frame bank)
    bank = synthetic.make_frame_bank(n1, n3, F, B, seed=0, world=world, rank=rank) if F else None
    nslots = args.slots or max(2, args.match_streams + 1)
    while F and not args.slots and F % nslots:
        nslots += 1
    m = matcher.from_state_dict(sd, {**synthetic.DEFAULT_HPARAMS,
                                     "attention_precision": args.precision})
    detector, images = None, None
    if args.e2e:
        from onepose_amd.superpoint import SuperPoint
        detector = SuperPoint({"nms_radius": 3, "keypoint_threshold": 0.005,
                               "max_keypoints": n1, "remove_borders": 4})
        detector.load_state_dict(synthetic.superpoint_state_dict(0))
        S = args.image_size
        images = np.stack([synthetic.superpoint_image(S, S, fs + i) for i in range(B)])
    pipe = FramePipeline(m, data["keypoints3d"][0], data["descriptors3d_db"][0],
                         data["descriptors2d_db"][0], B, n1, dev, scale=1000.0,
                         slots=nslots, detector=detector,
                         image_hw=(args.image_size, args.image_size),
                         object_cache=not args.no_object_cache, desc_dtype=args.desc_dtype)
    pipe.fused_pose = not args.unfused_pose
    pipe.pose_priority = args.pose_priority
    pipe.match_priority = args.match_priority
    cached = pipe.object_cache is not None
    pipe.set_frames(data["descriptors2d_query"], data["keypoints2d"],
                    np.stack([f.K for f in frames]), np.stack([f.pose_gt for f in frames]))
    if images is not None:
        pipe.set_images(images)
    if bank is not None:
        pipe.set_frame_bank(bank["descriptors2d_query"], bank["keypoints2d"], bank["K"],
                            bank["pose_gt"])

    # setup: one eager pass (loads every kernel's code object) before the profile pass; the W
    # warm-up steps run right before the timed region, below
    pipe.enqueue()
    torch.cuda.synchronize()

    # per-kernel profile pass (all kinds, HIP events, eager) to find the dominant kernel
    names = profile_kinds(lib)
    kinds, ms = run_profiled(lib, pipe, 3, (1 << len(names)) - 1, 4096)
    per_kind = {}
    for k, t in zip(kinds, ms):
        per_kind.setdefault(names[k], []).append(float(t))
    total = {k: sum(v) / 3.0 for k, v in per_kind.items()}
    mean_launch = {k: sum(v) / len(v) for k, v in per_kind.items()}
    # the dominant kernel is timed by device stamps, which the token GEMMs record
    dominant = max((k for k in total if kernel_work(k, B, n1, n3, L, cached) and k in STAMPED),
                   key=lambda k: total[k])
    dom_id = names.index(dominant)

    # Timed region: K steps; every step runs every kernel of the frame path.  With graphs
    # (default) the matcher stage and the pose stage are each one HIP-graph replay (captured
    # once per buffer slot before the timed region).  Default schedule: the pose stage of
    # step k (one workgroup per frame) overlaps the matcher of step k+1 on a second stream.
    overlap, graphs_on = not args.serial, not args.eager
    # stamping must be on while the graphs are captured (the accumulator address is a kernel
    # argument); begin_device again below re-zeroes the same accumulators
    sp_id = names.index("sp_conv")
    stamp_mask = (1 << dom_id) | ((1 << sp_id) if args.e2e else 0)
    if args.no_stamps:   # diagnostic: what device stamping costs the timed region
        stamp_mask = 0
    _lib.check(lib.onepose_profile_begin_device(stamp_mask), "profile_begin_device")
    # staged inputs (FramePipeline.prime_inputs): each pose stage ends with the input stage of
    # the step that next uses its slot, so the matcher's launch chain starts at its first layer
    staged = (overlap and pipe.staged_ok() and not args.no_staged_inputs
              and not args.diag_no_pose and not args.diag_steps)
    if not args.staged_split:
        # the pose streams' share of the forward that measured best on one box: with bf16
        # attention the layers take 0.33 ms per frame instead of 0.54, so a longer pose-stream
        # chain delays the slot's next matcher and only the winners move there
        args.staged_split = 15 if args.precision == "bf16" else 13
    if not args.staged_head:
        # self-attention 1's 2D half (a few small launches) ahead on the pose stream: +1-2% at
        # fp32 / split, +4% at config 5, but -11% for bf16 attention at config 2, whose 0.33 ms
        # layers leave the pose streams no room
        # (--e2e: the detector is staged with the inputs, and self-attention 1 ahead as well
        # loses, profiles/r06/e2e_staged)
        args.staged_head = (1 if args.e2e or (args.precision == "bf16" and n1 * n3 <= 1024 * 4096)
                            else 3)
    if staged:
        pipe.staged_split = args.staged_split
        pipe.staged_head = args.staged_head
    stage_graphs = (pipe.capture_stages(torch.cuda.graph_pool_handle(), staged=staged)
                    if graphs_on else None)
    if staged:
        pipe.prime_inputs()
    step_graph = pipe.capture(0) if graphs_on and not overlap else None

    step_events = []

    marks = []   # per step: events at matcher start / matcher done / pose done

    def run_steps(k, record=False):
        if args.diag_steps and k == args.steps:
            out = None
            for _ in range(k):
                out = run_steps(1)
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                step_events.append(ev)
            return out
        if overlap:
            pipe.run_stream(k, graphs=stage_graphs,
                            marks=marks if record and args.stage_marks else None,
                            match_streams=args.match_streams, pose=not args.diag_no_pose,
                            staged=staged,
                            pose_streams=args.pose_streams or args.match_streams)
            return pipe.slots[(k - 1) % len(pipe.slots)]
        for _ in range(k):
            if step_graph is not None:
                step_graph.replay()
            else:
                pipe.enqueue()
        return pipe.slots[0]

    frame_ids = torch.arange(fs, fe, dtype=torch.float64, device=dev)[:, None]
    # the bank's global frame indices go to the device here, not inside the timed region: a
    # pageable host -> device copy there would block the host until the K steps drained and
    # leave the result rows' launches to start on an idle GPU (~0.2 ms of a 20-step region)
    bank_gid = (torch.as_tensor(bank["frame_id"], dtype=torch.float64, device=dev)
                if bank is not None else None)

    def result_rows(slot):   # per-frame result row: pose, errors, cm/deg flags, inliers, status,
        # and the frame's index in the global batch (rank 0 checks the gathered order)
        if bank is not None:   # every bank entry's frames (the results of its last run)
            r = pipe.bank_results
            gid = bank_gid
            return torch.cat([r["pose"].reshape(F * B, 12), r["R_err"].reshape(-1, 1),
                              r["t_err"].reshape(-1, 1), r["cmd"].reshape(-1, 3).double(),
                              r["n_inliers"].reshape(-1, 1).double(),
                              r["status"].reshape(-1, 1).double(), gid.reshape(-1, 1)], 1)
        return torch.cat([slot.pose.reshape(B, 12), slot.R_err[:, None], slot.t_err[:, None],
                          slot.cmd.double(), slot.n_inliers[:, None].double(),
                          slot.status[:, None].double(), frame_ids], 1)

    n_rows = world * B * (F or 1)   # gathered result rows (global frames)

    # first replay of each graph (upload) and the first use of every torch kernel the timed
    # region launches (ROCm loads a kernel's code object lazily at its first launch, which
    # can take tens of ms) stay out of the timed region
    D.gather_frames(result_rows(run_steps(max(2, len(pipe.slots), F))), n_rows)
    torch.cuda.synchronize()
    # settle + W warm-up steps of the timed schedule, back to back and immediately before the
    # timed region: the GPU leaves its idle power state within them (after >= 20 ms idle a
    # 20-step region reads ~8% slow for its first milliseconds, tools/short_probe.py; after
    # only 5 busy steps still ~6%, tools/gpu_s20.sh)
    settle = max(0, args.settle_steps - args.warmup)
    if settle > 0:   # untimed, same schedule: the GPU's clock / power state settles
        run_steps(settle)
    if args.warmup > 0:
        run_steps(args.warmup)
    # the dominant kernel's launches are timed on the device (first workgroup start -> last
    # workgroup end), accumulated over every launch inside the timed region
    _lib.check(lib.onepose_profile_begin_device(stamp_mask), "profile_begin_device")
    if pg:
        pg.barrier()
    torch.cuda.synchronize()
    ev_begin = torch.cuda.Event(enable_timing=True)
    ev_end = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev_begin.record()
    last = run_steps(args.steps, record=True)
    host_enqueue = time.perf_counter() - t0   # host time to issue the K steps
    result = D.gather_frames(result_rows(last), n_rows)   # the only cross-rank exchange
    ev_end.record()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    nk = len(names)
    launches, tot_ms = np.zeros(nk, np.int64), np.zeros(nk, np.float64)
    _lib.check(lib.onepose_profile_end_device(launches.ctypes.data, tot_ms.ctypes.data, nk),
               "profile_end_device")
    alone_ms = float(mean_launch[dominant])
    n_dom = int(launches[dom_id])
    if args.no_stamps:
        n_dom, dom_ms = 0, alone_ms
    else:
        assert n_dom > 0 and tot_ms[dom_id] > 0, "dominant-kernel timing missing"
        dom_ms = float(tot_ms[dom_id] / n_dom)
    elapsed = D.max_over_ranks(elapsed, dev)   # the slowest rank's clock

    stage_ms = None
    if marks:   # matcher / pose stage GPU times over the timed region (diagnostic)
        mt = [a.elapsed_time(b) for a, b, _ in marks]
        pt = [b.elapsed_time(c) for _, b, c in marks]
        gap = [marks[i][1].elapsed_time(marks[i + 1][0]) for i in range(len(marks) - 1)]
        s2s = [marks[i][0].elapsed_time(marks[i + 1][0]) for i in range(len(marks) - 1)]
        # idle time of a match stream between its consecutive frames (frame i and i + m run on
        # the same stream; frame i + m waits for its buffer slot's previous pose stage)
        m_ = args.match_streams
        sgap = [marks[i][1].elapsed_time(marks[i + m_][0]) for i in range(len(marks) - m_)]
        stage_ms = {"gpu_region_ms": round(ev_begin.elapsed_time(ev_end), 3),
                    "lead_ms": round(ev_begin.elapsed_time(marks[0][0]), 3),
                    "tail_ms": round(marks[-1][2].elapsed_time(ev_end), 3),
                    "matcher_mean": round(float(np.mean(mt)), 4),
                    "gap_mean": round(float(np.mean(gap)), 4) if gap else None,
                    "gap_max": round(float(np.max(gap)), 4) if gap else None,
                    "step_mean": round(float(np.mean(s2s)), 4) if s2s else None,
                    "matcher_max": round(float(np.max(mt)), 4),
                    "pose_mean": round(float(np.mean(pt)), 4),
                    "pose_max": round(float(np.max(pt)), 4),
                    "stream_gap_mean": round(float(np.mean(sgap)), 4) if sgap else None,
                    "stream_gap_max": round(float(np.max(sgap)), 4) if sgap else None,
                    # per step, from the region's start: matcher start, matcher done, pose done
                    "per_step_ms": [[round(ev_begin.elapsed_time(e), 3) for e in m]
                                    for m in marks]}
    diag = []
    if step_events:
        diag.append([round(a.elapsed_time(b), 3) for a, b in zip(step_events, step_events[1:])])
    for _ in range(args.diag_repeats):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        run_steps(args.steps)
        torch.cuda.synchronize()
        diag.append(round((time.perf_counter() - t1) / args.steps * 1e3, 4))

    res = result.cpu().numpy()
    frames_total = world * B * args.steps
    det = None
    if args.e2e:
        S = args.image_size
        conv_ms = float(tot_ms[sp_id])
        conv_flop = superpoint_conv_flops(S, S) * B * args.steps
        counts = torch.cat([o.det_counts for o in pipe.slots]).cpu().numpy()
        det = {"image_hw": [S, S], "max_keypoints": n1,
               "keypoints_saturated": bool((counts == n1).all()),
               "conv_launches_timed": int(launches[sp_id]),
               "conv_ms_per_frame": round(conv_ms / (B * args.steps), 4),
               "conv_flop_per_frame": superpoint_conv_flops(S, S),
               "conv_achieved_tflops": round(conv_flop / (conv_ms * 1e-3) / 1e12, 2),
               "conv_frac_fp32_mfma": round(conv_flop / (conv_ms * 1e-3) / 1e12
                                            / FP32_MFMA_PEAK_TFLOPS, 4),
               "timing": "sum of SuperPoint MFMA-conv launch durations (device clock)"}
    value = frames_total / elapsed
    work, unit, bound = kernel_work(dominant, B, n1, n3, L, cached)
    achieved = work / (dom_ms * 1e-3) / 1e12
    bf_dom = args.precision == "bf16" and dominant in ("qkv_gemm", "mlp1_gemm", "mlp2_gemm")
    peak = BF16_MFMA_PEAK_TFLOPS if bf_dom else FP32_MFMA_PEAK_TFLOPS
    traffic, traffic_src = None, None
    if (B, n1, n3, L) == (1, 1024, 4096, 8) and args.precision == "fp32":
        traffic, traffic_src = pmc_traffic(dominant)
    elif (B, n1, n3, L) == (1, 2048, 8192, 8) and args.precision == "bf16":
        traffic, traffic_src = pmc_traffic(dominant + ("_bf16" if bf_dom else ""), "pmc_c5")
    roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak,
            "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
            "traffic": traffic, "traffic_unit": "HBM bytes per launch (PMC)",
            "traffic_source": traffic_src, "kernel": dominant,
            "avg_launch_us": round(dom_ms * 1e3, 2),
            "launches_timed": n_dom, "flop_per_launch": work,
            "timing": "device clock, first workgroup start to last workgroup end",
            # context: the same kernel when nothing else runs (serial profile pass before the
            # timed region, HIP events); inside the timed region a launch shares the chip with
            # the other match stream's kernels
            "alone": {"avg_launch_us": round(alone_ms * 1e3, 2),
                      "frac": round(work / (alone_ms * 1e-3) / 1e12 / peak, 4),
                      "timing": "serial profile pass (3 steps), HIP events per launch"}}

    # SURVEY.md §8d "fraction = F * frames/s / peak" for the whole frame's contractions
    ff = frame_flops(n1, n3, L, cached, B)
    formula = ("F_dep - 688128 n3 (object prefix and cross-attention 1's 3D half cached)"
               if cross_cached(cached, B) else "F_dep (object prefix cached)" if cached else "F")
    fx = executed_mfma_flops(n1, n3, cached)
    frame_roof = {"basis": "algorithmic (SURVEY.md section 8d)", "flop_per_frame": ff,
                  "formula": formula, "achieved_tflops": round(ff * value / 1e12, 2),
                  "peak": peak, "frac": round(ff * value / 1e12 / peak, 4),
                  "executed": {"mfma_flop_per_frame": fx,
                               "achieved_tflops": round(fx * value / 1e12, 2),
                               "frac": round(fx * value / 1e12 / peak, 4),
                               "note": "MFMA FLOPs the kernels execute (the Mf fold removes the "
                                       "merge conv and the attention apply)"}}

    # the gathered rows are the global frames (one object's sequence sharded over ranks); with
    # a bank, step j's global batch is frames [j world B, (j + 1) world B), and a row's weight is
    # the number of timed steps that ran its bank entry (step k runs entry k % F)
    pose_summary = summarize_pose(res, world, B, F, args.steps)
    if args.e2e:
        # Random-weight SuperPoint descriptors barely discriminate (cosine 0.97 between random
        # keypoints of the synthetic images; trained weights are not available offline), so the
        # synthetic object never matches the images' keypoints: the pose stage runs on every
        # frame, but on ~0 correspondences.  The frame rate includes its launches; its result
        # is not a pose measurement ("From images").
        pose_summary = {"status": "skipped", "reason": "no correspondences between random-weight "
                        "SuperPoint keypoints and the synthetic object; the pose stage still "
                        "runs every frame (its launches are timed)",
                        "n_inliers_mean": pose_summary["n_inliers_mean"],
                        "status_ok": pose_summary["status_ok"]}
    cfg_name = {(1024, 4096): "config 2", (1024, 16384): "config 3",
                (2048, 8192): "config 5"}.get((n1, n3), "custom")
    if args.precision == "bf16":
        cfg_name += " (bf16-MFMA attention)"
    elif args.precision == "fp32_split":
        cfg_name += " (fp32 attention as 3-piece bf16 split)"
    if args.desc_dtype == "fp16":
        cfg_name += " (fp16 desc)"
    if rank == 0:
        sched = (f"matchers of consecutive steps on {args.match_streams} concurrent stream(s), "
                 f"each step's pose stage on one of {args.pose_streams or args.match_streams} "
                 "pose stream(s) overlapping the next matchers"
                 if overlap else "serial steps")
        sched += "; stages replayed as HIP graphs" if graphs_on else "; host-launched kernels"
        tail_name = ({13: "final projection, score GEMM and dual-softmax winners",
                      14: "score GEMM and dual-softmax winners",
                      15: "dual-softmax winners"}.get(args.staged_split)
                     or f"GNN layers {args.staged_split - 1}-11, final projection, score GEMM "
                        "and dual-softmax winners")
        head_name = ("input stage" if args.staged_head <= 1 else
                     "input stage and self-attention 1's 2D half" if args.staged_head == 3 else
                     f"input stage and GNN layers 0-{args.staged_head - 2}")
        sched += ((f"; each step's matcher {head_name} run at the end of its slot's previous "
                   f"pose stage, its {tail_name} at the start of its own") if staged else "")
        sched += ("; object prefix (GAT 0 + 3D half of self-attention 1) prepared once per object"
                  if cached else "; every layer run per frame")
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "settle_steps": settle,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": {"fp32": "fp32",
                      "fp32_split": "fp32 (attention GEMMs as the exact 3-piece bf16 split on "
                                    "bf16 MFMA, fp32 accumulation)",
                      "bf16": "bf16 attention GEMMs, fp32 rest"}[args.precision]
                     + ("; descriptors fp16 in HBM (converted on load)"
                        if args.desc_dtype == "fp16" else ""),
            "data": "synthetic",
            "config": {"workload": (f"{cfg_name}: {n1} kpts x {n3} 3D pts, L={L}, {B} frame(s) per "
                                    f"GPU per step; "
                                    + (f"SuperPoint on {args.image_size}x{args.image_size} images + "
                                       if args.e2e else "")
                                    + f"matcher + RANSAC-EPnP + cm/deg; {sched}"),
                       "n1": n1, "n3": n3, "num_leaf": L, "batch_per_gpu": B,
                       "global_batch": n_global,
                       # frame buffer slots of the pipeline (a pipeline setting: rounds 1-4 ran 3,
                       # the 64-frame bank since round 5 gives 4 with two match streams)
                       "slots": nslots, "frame_bank": F,
                       # the staged schedule's stage split (onepose_match_cached_stages): the
                       # match streams run stages [head, split), the pose streams the rest
                       "staged": ({"head": args.staged_head, "split": args.staged_split}
                                  if staged else None),
                       "parallelism": f"frame-dp{world} (one object; global batch of "
                                      f"{n_global} frames sharded contiguously over ranks)"},
            "pose": pose_summary,
            "roofline": roof,
            "frame_roofline": frame_roof,
            **({"detector": det} if det else {}),
            "host_enqueue_ms_per_step": round(host_enqueue / args.steps * 1e3, 4),
            "library": {"path": os.path.relpath(_lib.LIB_PATH, REPO),
                        "overridden_by_ONEPOSE_LIB": bool(os.environ.get("ONEPOSE_LIB"))},
            **({"diagnostic": "pose stage skipped (--diag-no-pose): not the metric"}
               if args.diag_no_pose else {}),
            **({"stage_ms": stage_ms} if stage_ms else {}),
            "kernel_ms_per_step": {k: round(v, 4) for k, v in sorted(total.items(),
                                                                     key=lambda kv: -kv[1])},
            **({"diag_ms_per_step": diag} if diag else {}),
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(sd, data, frames, obj,
                                               detector_image=images[0] if args.e2e else None)
        print(json.dumps(out))
    if pg:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
