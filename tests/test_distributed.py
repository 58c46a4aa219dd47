"""Frame-sharded multi-rank path on CPU: world_size 2 over gloo (127.0.0.1).

Each rank solves the pose of its contiguous shard of frames (the C RANSAC-EPnP oracle stands
in for the GPU stage -- on the box the same helpers carry the HIP results), gathers the
per-frame result rows, and every rank must hold exactly what one process computes for all
frames, in frame order.  Uneven shards (7 frames on 2 ranks) and the max-over-ranks timer are
covered."""
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
