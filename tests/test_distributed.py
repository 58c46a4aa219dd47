"""Frame-sharded multi-rank path on CPU: world_size 2 over gloo (127.0.0.1).

Each rank solves the pose of its contiguous shard of frames (the C RANSAC-EPnP oracle stands
in for the GPU stage -- on the box the same helpers carry the HIP results), gathers the
per-frame result rows, and every rank must hold exactly what one process computes for all
frames, in frame order.  Uneven shards (7 frames on 2 ranks) and the max-over-ranks timer are
covered.  The bench's own sharding (one object's global batch, each rank its frame_shard slice
of one frame sequence, bench.py) is covered end to end with the CPU matcher oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from onepose_amd import distributed as D

N_FRAMES = 7


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def frame_rows(start, stop):
    from onepose_amd import synthetic as S
    from oracle import pnp_oracle as O
    rows = []
    for f in range(start, stop):
        rs = np.random.RandomState(100 + f)
        K = S.crop_intrinsics()
        R = S.random_rotation(rs)
        pose = np.concatenate([R, np.array([[0.01], [-0.02], [0.45]])], 1)
        pts = rs.uniform(-0.1, 0.1, (120, 3)).astype(np.float32)
        uv = (S.project(K, pose, pts.astype(np.float64)) + rs.normal(0, 0.5, (120, 2)))
        st, est, _, nin, _ = O.pnp_ransac(uv.astype(np.float32), pts * 1000.0, K, scale=1000.0)
        r_err, t_err = O.pose_error(est, pose)
        rows.append(np.concatenate([est.reshape(-1), [r_err, t_err, nin, st, f]]))
    return torch.tensor(np.array(rows).reshape(-1, 17), dtype=torch.float64)


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    assert D.init("gloo")
    s, e = D.frame_shard(N_FRAMES, world, rank)
    full = D.gather_frames(frame_rows(s, e), N_FRAMES)
    slowest = D.max_over_ranks(float(rank + 1))
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), full.numpy())
    np.save(os.path.join(out_dir, f"max{rank}.npy"), np.array([slowest]))
    dist.barrier()
    dist.destroy_process_group()


def test_frame_shard_covers_all_frames():
    for n in (0, 1, 7, 8, 256):
        for world in (1, 2, 3, 8):
            got = [D.frame_shard(n, world, r) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(got, got[1:]))


def test_gather_is_identity_without_a_group():
    t = torch.arange(6.0).reshape(3, 2)
    assert D.gather_frames(t, 3) is t


@pytest.mark.timeout(240)
def test_two_rank_gloo_gather_matches_single_process(tmp_path):
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    ref = frame_rows(0, N_FRAMES).numpy()
    for r in range(2):
        got = np.load(tmp_path / f"rank{r}.npy")
        np.testing.assert_array_equal(got, ref)
        assert float(np.load(tmp_path / f"max{r}.npy")[0]) == 2.0


# ---- the bench's sharding: one object's global batch, frame_shard slices, global order ----
N1, N3, LEAF, B_PER_RANK = 96, 160, 4, 3
N_GLOBAL = 2 * B_PER_RANK   # world 2


def shard_rows(world, rank):
    """What one bench rank computes (bench.py): the object from seed 0, its frame_shard slice of
    the global batch world * B, matcher (numpy oracle standing in for the HIP path) ->
    correspondences -> RANSAC-EPnP (C oracle) -> errors; rows end with the global frame index."""
    from onepose_amd import synthetic as S
    from oracle import matcher_np as M
    from oracle import pnp_oracle as O
    s, e = D.frame_shard(N_GLOBAL, world, rank)
    sd = S.make_state_dict(0)
    data, obj, frames = S.make_matcher_inputs(N1, N3, LEAF, seed=0, frame_ids=range(s, e))
    pred, _ = M.forward(sd, data)
    rows = []
    for i, f in enumerate(frames):
        # M.forward returns sample 0's correspondences (as the reference does): one frame a call
        one = {k: v[i:i + 1] for k, v in data.items()}
        p = pred if i == 0 else M.forward(sd, one)[0]
        m0 = p["matches0"].reshape(-1)
        ok = m0 > -1
        st, est, _, nin, _ = O.pnp_ransac(f.keypoints2d[ok].astype(np.float32),
                                          obj.keypoints3d[m0[ok]].astype(np.float32) * 1000.0,
                                          f.K, scale=1000.0)
        r_err, t_err = O.pose_error(est, f.pose_gt)
        rows.append(np.concatenate([est.reshape(-1), [r_err, t_err, nin, st, int(ok.sum()),
                                                     s + i]]))
    return torch.tensor(np.array(rows).reshape(-1, 18), dtype=torch.float64)


def _bench_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    assert D.init("gloo")
    full = D.gather_frames(shard_rows(world, rank), N_GLOBAL)
    np.save(os.path.join(out_dir, f"bench{rank}.npy"), full.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_bench_shards_one_objects_batch(tmp_path):
    """world 2 x B 3: the gathered rows equal one process running the whole 6-frame batch of
    the same object, in global frame order, and the frames are not all alike (distinct poses)."""
    port = _free_port()
    mp.start_processes(_bench_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    ref = shard_rows(1, 0)   # world 1: all 6 frames in one process
    assert ref.shape[0] == N_GLOBAL
    for r in range(2):
        got = np.load(tmp_path / f"bench{r}.npy")
        np.testing.assert_array_equal(got, ref.numpy())
        np.testing.assert_array_equal(got[:, -1], np.arange(N_GLOBAL))
    assert (ref[:, 16] > 20).all()                       # every frame has correspondences
    assert len({tuple(np.round(r[:12], 6)) for r in ref.numpy()}) == N_GLOBAL


# ---- the bench's frame bank: F steps of distinct frames, step k runs entry k % F ----
def test_frame_bank_shards_one_sequence():
    """Rank r's bank entry (j, i) is global frame (j world + r) B + i: the ranks' banks together
    are the world-1 bank of batch world * B, frame for frame."""
    from onepose_amd import synthetic as S
    world, B, F = 2, 2, 3
    one = S.make_frame_bank(N1, N3, F, world * B, seed=0)
    for r in range(world):
        bank = S.make_frame_bank(N1, N3, F, B, seed=0, world=world, rank=r)
        for j in range(F):
            for i in range(B):
                g = bank["frame_id"][j, i]
                assert g == (j * world + r) * B + i
                jj, ii = divmod(int(g), world * B)
                assert one["frame_id"][jj, ii] == g
                np.testing.assert_array_equal(bank["keypoints2d"][j, i], one["keypoints2d"][jj, ii])
                np.testing.assert_array_equal(bank["descriptors2d_query"][j, i],
                                              one["descriptors2d_query"][jj, ii])
                np.testing.assert_array_equal(bank["pose_gt"][j, i], one["pose_gt"][jj, ii])
    # distinct frames
    assert len({tuple(np.round(p.reshape(-1), 6)) for p in one["pose_gt"].reshape(-1, 3, 4)}) == F * world * B


def test_bench_pose_summary_weights_every_timed_frame():
    """summarize_pose: a row counts once per timed step that ran its bank entry; rows may come
    in any order (the gather is in rank order, not frame order)."""
    import bench
    world, B, F, steps = 2, 2, 4, 10
    n = world * B * F
    res = np.zeros((n, 20))
    res[:, 19] = np.arange(n)
    res[:, 12] = np.arange(n)          # R_err = global frame id
    res[:, 14] = (np.arange(n) % 2)    # cmd1
    res[:, 18] = 0
    perm = np.random.RandomState(0).permutation(n)
    s = bench.summarize_pose(res[perm], world, B, F, steps)
    w = np.bincount(np.arange(steps) % F, minlength=F)[np.arange(n) // (world * B)]
    assert s["frames"] == world * B * steps == w.sum()
    assert s["distinct_frames"] == n
    assert abs(s["R_err_deg_mean"] - (w * np.arange(n)).sum() / w.sum()) < 1e-12
    assert abs(s["cmd1"] - (w * (np.arange(n) % 2)).sum() / w.sum()) < 1e-12
    s1 = bench.summarize_pose(res[:world * B], world, B, 0, steps)   # no bank: one batch
    assert s1["frames"] == world * B
