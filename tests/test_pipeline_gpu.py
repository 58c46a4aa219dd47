"""The per-frame pipeline (matcher -> selection -> RANSAC-EPnP -> cm/deg) gives bit-identical
results whether its launches come from the host, from a replayed HIP graph, or from the
two-stream overlapped schedule -- and a captured graph picks up new frames written into the
pipeline's static input buffers."""
import numpy as np
import pytest
import torch

from onepose_amd import matcher, synthetic
from onepose_amd.pipeline import FramePipeline
from parity import assert_pred_equal

N1, N3, L, B = 256, 1024, 8, 2


def _outputs(slot):
    return {k: getattr(slot, k).cpu().numpy().copy()
            for k in ("matches0", "matches1", "mscores0", "pose", "inlier_mask", "n_inliers",
                      "status", "R_err", "t_err", "cmd")}


def _assert_same(a, b):
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


@pytest.fixture(scope="module")
def setup():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    dev = torch.device("cuda", 0)
    sd = synthetic.make_state_dict(0)
    data, obj, frames = synthetic.make_matcher_inputs(N1, N3, L, seed=5, batch=2 * B)
    m = matcher.from_state_dict(sd)
    pipe = FramePipeline(m, data["keypoints3d"][0], data["descriptors3d_db"][0],
                         data["descriptors2d_db"][0], B, N1, dev, scale=1000.0, slots=3)
    Ks = np.stack([f.K for f in frames])
    gts = np.stack([f.pose_gt for f in frames])
    batches = [(data["descriptors2d_query"][i:i + B], data["keypoints2d"][i:i + B],
                Ks[i:i + B], gts[i:i + B]) for i in (0, B)]
    return pipe, batches


@pytest.mark.gpu
def test_graph_replay_matches_eager(setup):
    pipe, batches = setup
    eager = []
    for bt in batches:
        pipe.set_frames(*bt)
        pipe.enqueue(0)
        torch.cuda.synchronize()
        eager.append(_outputs(pipe.slots[0]))
    assert eager[0]["status"].tolist() == [0] * B

    pipe.set_frames(*batches[0])
    g = pipe.capture(0)
    for i, bt in enumerate(batches + batches):
        pipe.set_frames(*bt)          # new frame data into the captured buffers
        g.replay()
        torch.cuda.synchronize()
        _assert_same(eager[i % 2], _outputs(pipe.slots[0]))


@pytest.mark.gpu
def test_conf_needs_with_conf(setup):
    """with_conf=False (the default): conf_matrix is not kept, and reading it says so."""
    pipe, _ = setup
    with pytest.raises(RuntimeError, match="with_conf=True"):
        pipe.conf


@pytest.mark.gpu
def test_fused_pose_stage_matches_separate_calls(setup):
    """onepose_pose_stage (selection in the RANSAC kernel, errors in the refit kernel) gives
    the bits of onepose_select_correspondences + onepose_pnp_ransac + onepose_pose_errors."""
    pipe, batches = setup
    for bt in batches:
        pipe.set_frames(*bt)
        pipe.enqueue_front(0)
        pipe.enqueue_pose(0, fused=False)
        torch.cuda.synchronize()
        sep = _outputs(pipe.slots[0])
        sep.update(pts2d=pipe.slots[0].pts2d.cpu().numpy().copy(),
                   pts3d=pipe.slots[0].pts3d.cpu().numpy().copy(),
                   counts=pipe.slots[0].counts.cpu().numpy().copy())
        for k in ("pose", "inlier_mask", "R_err", "t_err", "cmd", "n_inliers", "counts"):
            getattr(pipe.slots[0], k).zero_()
        pipe.enqueue_pose(0, fused=True)
        torch.cuda.synchronize()
        fused = _outputs(pipe.slots[0])
        o = pipe.slots[0]
        for b in range(B):
            c = int(sep["counts"][b])
            assert int(o.counts[b]) == c
            np.testing.assert_array_equal(o.pts2d[b, :c].cpu().numpy(), sep["pts2d"][b, :c])
            np.testing.assert_array_equal(o.pts3d[b, :c].cpu().numpy(), sep["pts3d"][b, :c])
        _assert_same(sep_core := {k: sep[k] for k in fused}, fused)
        assert sep_core["status"].tolist() == [0] * B


@pytest.mark.gpu
def test_stream_schedule_matches_eager(setup):
    pipe, batches = setup
    pipe.set_frames(*batches[1])
    pipe.enqueue(0)
    torch.cuda.synchronize()
    ref = _outputs(pipe.slots[0])
    pipe.run_stream(5)
    torch.cuda.synchronize()
    for s in pipe.slots:
        _assert_same(ref, _outputs(s))


@pytest.mark.gpu
def test_stream_schedule_with_stage_graphs_matches_eager(setup):
    pipe, batches = setup
    pipe.set_frames(*batches[0])
    pipe.enqueue(0)
    torch.cuda.synchronize()
    ref = _outputs(pipe.slots[0])
    graphs = pipe.capture_stages()
    pipe.run_stream(7, graphs=graphs)
    torch.cuda.synchronize()
    for s in pipe.slots:
        _assert_same(ref, _outputs(s))


@pytest.mark.gpu
def test_two_concurrent_matcher_streams_match_eager(setup):
    """Consecutive frames' matchers on two streams (graphs), pose on a third: same bits."""
    pipe, batches = setup
    pipe.set_frames(*batches[1])
    pipe.enqueue(0)
    torch.cuda.synchronize()
    ref = _outputs(pipe.slots[0])
    graphs = pipe.capture_stages()
    pipe.run_stream(9, graphs=graphs, match_streams=2)
    torch.cuda.synchronize()
    for s in pipe.slots:
        _assert_same(ref, _outputs(s))


@pytest.mark.gpu
def test_two_pose_streams_match_eager(setup):
    """Two matcher streams and two pose streams (the bench's default schedule): consecutive
    frames' pose stages run side by side on their own slots' buffers -- same bits."""
    pipe, batches = setup
    pipe.set_frames(*batches[1])
    pipe.enqueue(0)
    torch.cuda.synchronize()
    ref = _outputs(pipe.slots[0])
    graphs = pipe.capture_stages()
    pipe.run_stream(10, graphs=graphs, match_streams=2, pose_streams=2)
    torch.cuda.synchronize()
    for s in pipe.slots:
        _assert_same(ref, _outputs(s))


@pytest.mark.gpu
def test_frame_bank_runs_each_entry_like_eager():
    """A frame bank of F steps (bench.py --frames): step k runs entry k % F through its own
    captured graphs on slot k % slots; every entry's result rows equal an eager run of the
    same frames through the static inputs, bit for bit, under the bench's two-stream
    schedule."""
    dev = torch.device("cuda", 0)
    F = 3
    sd = synthetic.make_state_dict(0)
    data, obj, frames = synthetic.make_matcher_inputs(N1, N3, L, seed=5, batch=F * B)
    m = matcher.from_state_dict(sd)
    pipe = FramePipeline(m, data["keypoints3d"][0], data["descriptors3d_db"][0],
                         data["descriptors2d_db"][0], B, N1, dev, scale=1000.0, slots=3)
    Ks = np.stack([f.K for f in frames]).reshape(F, B, 3, 3)
    gts = np.stack([f.pose_gt for f in frames]).reshape(F, B, 3, 4)
    d2 = data["descriptors2d_query"].reshape(F, B, 256, N1)
    k2 = data["keypoints2d"].reshape(F, B, N1, 2)
    ref = []
    for j in range(F):
        pipe.set_frames(d2[j], k2[j], Ks[j], gts[j])
        pipe.enqueue(0)
        torch.cuda.synchronize()
        ref.append(_outputs(pipe.slots[0]))
    pipe.set_frame_bank(d2, k2, Ks, gts)
    with pytest.raises(ValueError):
        FramePipeline.set_frame_bank(pipe, d2[:2], k2[:2], Ks[:2], gts[:2])   # 2 % 3 slots
    graphs = pipe.capture_stages()
    assert len(graphs) == F
    pipe.run_stream(7, graphs=graphs, match_streams=2, pose_streams=2)
    torch.cuda.synchronize()
    r = pipe.bank_results
    for j in range(F):
        for k in ("pose", "R_err", "t_err", "cmd", "n_inliers", "status"):
            np.testing.assert_array_equal(r[k][j].cpu().numpy(), ref[j][k], err_msg=f"{k} {j}")
    assert len({tuple(np.round(x.reshape(-1), 6)) for x in r["pose"].cpu().numpy().reshape(-1, 12)}) == F * B
    # eager steps over the bank too
    for v in r.values():
        v.zero_()
    pipe.run_stream(F, match_streams=2)
    torch.cuda.synchronize()
    for j in range(F):
        np.testing.assert_array_equal(r["pose"][j].cpu().numpy(), ref[j]["pose"])


@pytest.mark.gpu
def test_frame_bank_staged_inputs_match_eager():
    """Staged stages (bench.py's default): the matcher's input stage runs at the end of the
    slot's previous pose stage and its tail (final projection, score GEMM, winners) at the start
    of its own pose stage (onepose_match_cached_stages); the step counter carries over between
    run_stream calls.  Consecutive stage ranges give the bits of the one-call forward, and every
    bank entry's result rows equal an eager run of its frames."""
    dev = torch.device("cuda", 0)
    F, n = 6, 3
    sd = synthetic.make_state_dict(0)
    data, obj, frames = synthetic.make_matcher_inputs(N1, N3, L, seed=11, batch=F * B)
    m = matcher.from_state_dict(sd)
    pipe = FramePipeline(m, data["keypoints3d"][0], data["descriptors3d_db"][0],
                         data["descriptors2d_db"][0], B, N1, dev, scale=1000.0, slots=n)
    Ks = np.stack([f.K for f in frames]).reshape(F, B, 3, 3)
    gts = np.stack([f.pose_gt for f in frames]).reshape(F, B, 3, 4)
    d2 = data["descriptors2d_query"].reshape(F, B, 256, N1)
    k2 = data["keypoints2d"].reshape(F, B, N1, 2)
    ref = []
    for j in range(F):
        pipe.set_frames(d2[j], k2[j], Ks[j], gts[j])
        pipe.enqueue(0)
        torch.cuda.synchronize()
        ref.append(_outputs(pipe.slots[0]))
    pipe.set_frame_bank(d2, k2, Ks, gts)
    with pytest.raises(RuntimeError, match="prime_inputs"):
        pipe.run_stream(1, staged=True)
    # the stages against the one-call forward, on the library's outputs directly
    o = pipe.slots[1]
    keys = ("matches0", "matches1", "mscores0", "mscores1")
    for j in (0, 4):
        pipe.enqueue_match(1, j)
        torch.cuda.synchronize()
        whole = {k: getattr(o, k).cpu().numpy().copy() for k in keys}
        for split in ([(0, 0), (1, 12), (13, 13), (14, 14), (15, 15)],
                      [(0, 5), (6, 12), (13, 15)], [(0, 1), (2, 2), (3, 3), (4, 11), (12, 15)],
                      [(0, 13), (14, 15)], [(0, 15)]):
            for k in keys:
                getattr(o, k).fill_(7)
            for rng in split:
                pipe.enqueue_match(1, j, stages=rng)
            torch.cuda.synchronize()
            for k in keys:
                np.testing.assert_array_equal(getattr(o, k).cpu().numpy(), whole[k],
                                              err_msg=f"{k} {split}")
    graphs = pipe.capture_stages(staged=True)
    pipe.prime_inputs()
    pipe.run_stream(7, graphs=graphs, match_streams=2, pose_streams=2, staged=True)
    pipe.run_stream(5, graphs=graphs, match_streams=2, pose_streams=2, staged=True)
    torch.cuda.synchronize()
    assert pipe._next_step == 12
    r = pipe.bank_results
    for j in range(F):
        for k in ("pose", "R_err", "t_err", "cmd", "n_inliers", "status"):
            np.testing.assert_array_equal(r[k][j].cpu().numpy(), ref[j][k], err_msg=f"{k} {j}")
    # host-launched staged steps continue the same bank sequence
    for v in r.values():
        v.zero_()
    pipe.run_stream(F, match_streams=2, staged=True)
    torch.cuda.synchronize()
    for j in range(F):
        np.testing.assert_array_equal(r["pose"][j].cpu().numpy(), ref[j]["pose"])
    # a one-call forward on a slot (or an unstaged run) drops the staged inputs: staged steps
    # need priming again
    pipe.enqueue_match(0, 0)
    with pytest.raises(RuntimeError, match="prime_inputs"):
        pipe.run_stream(1, graphs=graphs, staged=True)
    pipe.prime_inputs()
    pipe.run_stream(1, match_streams=2)
    with pytest.raises(RuntimeError, match="prime_inputs"):
        pipe.run_stream(1, graphs=graphs, staged=True)
    # the last two GNN layers on the pose stream too (bench.py --staged-split 11)
    pipe.staged_split = 11
    pipe.prime_inputs()
    with pytest.raises(ValueError, match="staged_split"):
        pipe.run_stream(1, graphs=graphs, staged=True)   # graphs of the other split
    graphs = pipe.capture_stages(staged=True)
    pipe.prime_inputs()
    for v in r.values():
        v.zero_()
    pipe.run_stream(F + 1, graphs=graphs, match_streams=2, pose_streams=2, staged=True)
    torch.cuda.synchronize()
    for j in range(F):
        for k in ("pose", "R_err", "t_err", "cmd", "n_inliers", "status"):
            np.testing.assert_array_equal(r[k][j].cpu().numpy(), ref[j][k], err_msg=f"{k} {j}")
    # self-attention 1 run ahead with the input stage (bench.py --staged-head 3)
    pipe.staged_split, pipe.staged_head = 13, 3
    graphs = pipe.capture_stages(staged=True)
    pipe.prime_inputs()
    for v in r.values():
        v.zero_()
    pipe.run_stream(F + 2, graphs=graphs, match_streams=2, pose_streams=2, staged=True)
    pipe.run_stream(F - 1, match_streams=2, staged=True)   # host-launched, continuing
    torch.cuda.synchronize()
    for j in range(F):
        for k in ("pose", "R_err", "t_err", "cmd", "n_inliers", "status"):
            np.testing.assert_array_equal(r[k][j].cpu().numpy(), ref[j][k], err_msg=f"{k} {j}")


@pytest.mark.gpu
@pytest.mark.parametrize("precision,desc,split,head", [("bf16", "fp16", 15, 3),
                                                        ("bf16", "fp16", 15, 1),
                                                        ("fp32_split", "fp32", 13, 3),
                                                        ("bf16", "fp32", 13, 1)])
def test_staged_stages_other_precisions(precision, desc, split, head):
    """The bench's staged schedules of the other lines (bf16 attention with only the winners on
    the pose stream, config 5's fp16 descriptors; the split mode from the final projection): the
    stage ranges give the one-call bits and every bank entry equals an eager run."""
    from onepose_amd import synthetic as S
    dev = torch.device("cuda", 0)
    F, n = 3, 3
    sd = S.make_state_dict(0)
    data, obj, frames = S.make_matcher_inputs(N1, N3, L, seed=13, batch=F * B)
    m = matcher.from_state_dict(sd, dict(S.DEFAULT_HPARAMS, attention_precision=precision))
    pipe = FramePipeline(m, data["keypoints3d"][0], data["descriptors3d_db"][0],
                         data["descriptors2d_db"][0], B, N1, dev, scale=1000.0, slots=n,
                         desc_dtype=desc)
    Ks = np.stack([f.K for f in frames]).reshape(F, B, 3, 3)
    gts = np.stack([f.pose_gt for f in frames]).reshape(F, B, 3, 4)
    d2 = data["descriptors2d_query"].reshape(F, B, 256, N1)
    k2 = data["keypoints2d"].reshape(F, B, N1, 2)
    ref = []
    for j in range(F):
        pipe.set_frames(d2[j], k2[j], Ks[j], gts[j])
        pipe.enqueue(0)
        torch.cuda.synchronize()
        ref.append(_outputs(pipe.slots[0]))
    pipe.set_frame_bank(d2, k2, Ks, gts)
    o = pipe.slots[1]
    keys = ("matches0", "matches1", "mscores0", "mscores1")
    pipe.enqueue_match(1, 2)
    torch.cuda.synchronize()
    whole = {k: getattr(o, k).cpu().numpy().copy() for k in keys}
    for k in keys:
        getattr(o, k).fill_(7)
    for rng in [(0, 0), (1, split - 1), (split, 15)]:
        pipe.enqueue_match(1, 2, stages=rng)
    torch.cuda.synchronize()
    for k in keys:
        np.testing.assert_array_equal(getattr(o, k).cpu().numpy(), whole[k], err_msg=k)
    pipe.staged_split, pipe.staged_head = split, head
    graphs = pipe.capture_stages(staged=True)
    pipe.prime_inputs()
    pipe.run_stream(2 * F + 1, graphs=graphs, match_streams=2, pose_streams=2, staged=True)
    torch.cuda.synchronize()
    r = pipe.bank_results
    for j in range(F):
        for k in ("pose", "R_err", "t_err", "cmd", "n_inliers", "status"):
            np.testing.assert_array_equal(r[k][j].cpu().numpy(), ref[j][k], err_msg=f"{k} {j}")


@pytest.mark.gpu
def test_detector_pipeline_from_images():
    """Images -> SuperPoint -> matcher -> selection -> RANSAC-EPnP: the detector stage writes
    exactly what SuperPoint.detect_raw returns, the matcher stage equals the module forward on
    those keypoints, and graph replay / two matcher streams reproduce the eager results."""
    from onepose_amd.superpoint import SuperPoint
    dev = torch.device("cuda", 0)
    n1, hw = 256, (256, 256)
    sp = SuperPoint({"nms_radius": 3, "max_keypoints": n1})
    sp.load_state_dict(synthetic.superpoint_state_dict(0))
    sp.to(dev)
    sd = synthetic.make_state_dict(0)
    data, obj, frames = synthetic.make_matcher_inputs(n1, N3, L, seed=6, batch=1)
    m = matcher.from_state_dict(sd)
    pipe = FramePipeline(m, data["keypoints3d"][0], data["descriptors3d_db"][0],
                         data["descriptors2d_db"][0], B, n1, dev, scale=1000.0, slots=3,
                         detector=sp, image_hw=hw)
    imgs = np.stack([synthetic.superpoint_image(*hw, s) for s in (10, 11)])
    pipe.set_images(imgs)
    pipe.K.copy_(torch.as_tensor(frames[0].K).expand_as(pipe.K))
    pipe.pose_gt.copy_(torch.as_tensor(frames[0].pose_gt)[:3].expand_as(pipe.pose_gt))
    pipe.enqueue(0)
    torch.cuda.synchronize()
    o = pipe.slots[0]
    assert o.det_counts.tolist() == [n1] * B
    raw = sp.detect_raw(torch.from_numpy(imgs)[:, None].to(dev))
    np.testing.assert_array_equal(o.kpts2d.cpu().numpy(), raw["keypoints"].cpu().numpy())
    np.testing.assert_array_equal(o.desc2d.cpu().numpy(), raw["descriptors"].cpu().numpy())
    d3 = torch.as_tensor(data["descriptors3d_db"][0]).to(dev)[None]
    db = torch.as_tensor(data["descriptors2d_db"][0]).to(dev)[None]
    k3 = torch.as_tensor(data["keypoints3d"][0]).to(dev)[None]
    for i in range(B):   # the module returns one frame's matches (GATs_SuperGlue.py:269-273)
        pred, _ = m({"keypoints2d": raw["keypoints"][i:i + 1], "keypoints3d": k3,
                     "descriptors2d_query": raw["descriptors"][i:i + 1],
                     "descriptors3d_db": d3, "descriptors2d_db": db})
        np.testing.assert_array_equal(o.matches0[i].cpu().numpy(),
                                      pred["matches0"].cpu().numpy())
    ref = _outputs(o)
    graphs = pipe.capture_stages()
    pipe.run_stream(6, graphs=graphs, match_streams=2)
    torch.cuda.synchronize()
    for s in pipe.slots:
        _assert_same(ref, _outputs(s))
    # staged: each slot's detector + input stage (+ self-attention 1) at the end of the slot's
    # previous pose stage, the tail on the frame's own pose stream (bench.py --e2e)
    for head in (1, 3):
        pipe.staged_split, pipe.staged_head = 13, head
        graphs = pipe.capture_stages(staged=True)
        pipe.prime_inputs()
        for s in pipe.slots:
            for k in ("pose", "matches0", "n_inliers"):
                getattr(s, k).zero_()
        pipe.run_stream(7, graphs=graphs, match_streams=2, pose_streams=2, staged=True)
        pipe.run_stream(2, match_streams=2, pose_streams=2, staged=True)   # host-launched
        torch.cuda.synchronize()
        for s in pipe.slots:
            _assert_same(ref, _outputs(s))


@pytest.mark.gpu
def test_device_stamps_count_and_time_graph_launches(setup):
    """bench.py's roofline timing (onepose_profile_begin_device): every MLP-conv-1 launch of a
    replayed graph is booked once, and the stamped average (first wave start to last wave end)
    agrees with HIP-event timing of the same launches run eagerly."""
    import ctypes
    from onepose_amd import _lib
    lib = _lib.load()
    pipe, batches = setup
    pipe.set_frames(*batches[0])
    names = [lib.onepose_profile_kind_name(i).decode() for i in range(64)
             if lib.onepose_profile_kind_name(i)]
    k = names.index("mlp1_gemm")
    # eager HIP-event reference
    _lib.check(lib.onepose_profile_begin(1 << k, 256), "profile_begin")
    for _ in range(4):
        pipe.enqueue(0)
    kinds = np.zeros(256, np.int32)
    ms = np.zeros(256, np.float32)
    cnt = np.zeros(1, np.int32)
    _lib.check(lib.onepose_profile_end(kinds.ctypes.data, ms.ctypes.data, 256, cnt.ctypes.data),
               "profile_end")
    per_frame = int(cnt[0]) // 4
    assert per_frame == 8
    ev_ms = float(ms[:cnt[0]].mean())
    # stamped graph replays
    _lib.check(lib.onepose_profile_begin_device(1 << k), "profile_begin_device")
    g = pipe.capture(0)
    _lib.check(lib.onepose_profile_begin_device(1 << k), "profile_begin_device")   # re-arm
    reps = 20
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    n = len(names)
    launches = np.zeros(n, np.int64)
    tot = np.zeros(n, np.float64)
    _lib.check(lib.onepose_profile_end_device(launches.ctypes.data, tot.ctypes.data, n),
               "profile_end_device")
    assert launches[k] == reps * per_frame
    st_ms = tot[k] / launches[k]
    assert 0.5 * ev_ms < st_ms < 1.5 * ev_ms, (st_ms, ev_ms)


@pytest.mark.gpu
@pytest.mark.parametrize("n1,n3,seed", [(256, 1024, 3), (1024, 4096, 4)])
def test_pipeline_frame_matches_oracle(n1, n3, seed):
    """The bench's per-frame path exactly as it runs there -- object cache (GAT 0, self-
    attention 1's and cross-attention 1's 3D halves, GAT leaf logits), cached matcher, fused
    selection + RANSAC-EPnP + cm/deg stage -- against the CPU oracle: the numpy matcher
    (GATs_SuperGlue.py:203-278; indices exact, tests/parity.py) and the C restatement of solvePnPRansac(EPNP) + query_pose_error on
    the pipeline's own correspondences (eval_utils.py:18-63; status and inliers exact, pose
    within 1e-6, the errors of that pose within 1e-6)."""
    from oracle import matcher_np as M
    from oracle import pnp_oracle as O
    dev = torch.device("cuda", 0)
    sd = synthetic.make_state_dict(0)
    data, _, frames = synthetic.make_matcher_inputs(n1, n3, L, seed=seed, batch=1)
    m = matcher.from_state_dict(sd)
    pipe = FramePipeline(m, data["keypoints3d"][0], data["descriptors3d_db"][0],
                         data["descriptors2d_db"][0], 1, n1, dev, scale=1000.0, slots=3)
    assert pipe.object_cache is not None
    pipe.set_frames(data["descriptors2d_query"], data["keypoints2d"], frames[0].K[None],
                    frames[0].pose_gt[None])
    pipe.enqueue(0)
    torch.cuda.synchronize()
    o = pipe.slots[0]
    got = o.matches0.cpu().numpy()[0]
    opred, oconf = M.forward(sd, data)
    # (pred holds batch element 0, GATs_SuperGlue.py:270-273)
    assert_pred_equal({"matches0": got, "matches1": o.matches1.cpu().numpy()[0],
                       "matching_scores0": o.mscores0.cpu().numpy()[0],
                       "matching_scores1": o.mscores1.cpu().numpy()[0]}, opred, "pipeline")
    assert (got > -1).sum() > 0.3 * n1
    n = int(o.counts.cpu()[0])
    assert n == int((got > -1).sum())
    st, pose, mask, nin, _ = O.pnp_ransac(o.pts2d.cpu().numpy()[0, :n], o.pts3d.cpu().numpy()[0, :n],
                                          frames[0].K, scale=1000.0)
    assert st == int(o.status.cpu()[0]) == 0
    assert nin == int(o.n_inliers.cpu()[0])
    gpose = o.pose.cpu().numpy()[0]
    np.testing.assert_allclose(gpose, pose, atol=1e-6)
    # the cm / deg errors of the frame's own pose (arccos near 0 deg would magnify the 1e-6
    # pose tolerance)
    r_err, t_err = O.pose_error(gpose, frames[0].pose_gt)
    np.testing.assert_allclose(o.R_err.cpu().numpy()[0], r_err, atol=1e-6)
    np.testing.assert_allclose(o.t_err.cpu().numpy()[0], t_err, atol=1e-6)
