"""onepose_match_sharded on the GPU: two (and three) ranks of a gloo group on one device, each
holding a contiguous shard of the object's 3D points, exchange the per-layer partials through
the all-gather callback; every rank must end with the whole frame's matches, equal to the
single-process GPU matcher on the unsplit frame (indices exactly except on low-margin rows,
scores to 2e-5) -- and equal to each other bitwise.  n3 = 5377 over 2 ranks gives shards of
2689 / 2688 points, either side of the 64-row QKV tile's threshold (43 x 6 = 258 vs 252 tiles):
every rank takes its tiles from the largest shard so the replicated 2D state rounds alike."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from parity import assert_pred_equal

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs(n1, n3, seed):
    from onepose_amd import synthetic
    sd = synthetic.make_state_dict(0)
    data, _, _ = synthetic.make_matcher_inputs(n1, n3, 8, seed=seed, batch=1)
    return sd, data


def _worker(rank, world, port, out_dir, n1, n3, seed, precision):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from onepose_amd import matcher, synthetic
    from onepose_amd.sharded import ShardedMatcher
    dev = torch.device("cuda", 0)
    sd, data = _inputs(n1, n3, seed)
    m = matcher.from_state_dict(sd, {**synthetic.DEFAULT_HPARAMS, "attention_precision": precision})
    sm = ShardedMatcher(m, data["keypoints3d"][0], data["descriptors3d_db"][0],
                        data["descriptors2d_db"][0], n1, dev)
    d2 = torch.from_numpy(data["descriptors2d_query"]).to(dev)
    m0, m1, s0, s1 = sm.match(d2)
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), m0=m0.cpu().numpy(), m1=m1.cpu().numpy(),
             s0=s0.cpu().numpy(), s1=s1.cpu().numpy())
    if rank == 0:   # the whole frame in one process
        inp = {k: torch.from_numpy(v).to(dev) for k, v in data.items()}
        pred, conf = m(inp)
        np.savez(os.path.join(out_dir, "whole.npz"), m0=pred["matches0"].cpu().numpy(),
                 m1=pred["matches1"].cpu().numpy(), s0=pred["matching_scores0"].cpu().numpy(),
                 s1=pred["matching_scores1"].cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,n1,n3", [(2, 256, 1024), (3, 200, 1023), (2, 512, 5377)])
def test_sharded_frame_equals_whole_frame(tmp_path, world, n1, n3):
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), n1, n3, 7, "fp32"),
                       nprocs=world, join=True, start_method="spawn")
    whole = np.load(tmp_path / "whole.npz")
    ranks = [np.load(tmp_path / f"r{r}.npz") for r in range(world)]
    for r in ranks[1:]:   # every rank holds the same whole-frame answer
        for k in ("m0", "m1", "s0", "s1"):
            np.testing.assert_array_equal(r[k], ranks[0][k])
    got = ranks[0]
    assert_pred_equal({"matches0": got["m0"][0], "matches1": got["m1"][0],
                       "matching_scores0": got["s0"][0], "matching_scores1": got["s1"][0]},
                      {"matches0": whole["m0"], "matches1": whole["m1"],
                       "matching_scores0": whole["s0"], "matching_scores1": whole["s1"]},
                      f"sharded over {world}")
    assert (got["m0"][0] > -1).sum() > 40
