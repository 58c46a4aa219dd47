"""RCCL on the device (torch.distributed backend "nccl" = RCCL on ROCm), world size 1: the
multi-GPU code paths bench.py and ShardedMatcher run at N > 1, executed through real RCCL
collectives on the one GPU a test box has (RCCL refuses two ranks on one device, so N > 1 is
covered by the gloo tests, tests/test_distributed.py and tests/test_sharded_gpu.py).
  * onepose_amd.distributed.gather_frames (dist.all_gather of the per-frame result rows) and
    max_over_ranks (dist.all_reduce MAX), as bench.py calls them;
  * ShardedMatcher with its RCCL all_gather_into_tensor callback on the matcher's stream, against
    the whole-frame matcher (tests/parity.py contract: the sharded path folds KV with kv_reduce +
    m_fold instead of kv_fold, so only the summation order differs).
The worker is spawned (start_method "spawn", as tests/test_sharded_gpu.py), so RCCL state never
enters the pytest process."""
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


def _worker(rank, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="1", RANK="0",
                      LOCAL_RANK="0")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from onepose_amd import distributed as D
    from onepose_amd import matcher, synthetic
    from onepose_amd.sharded import ShardedMatcher
    out = {"backend": dist.get_backend()}
    rows = torch.arange(5 * 19, dtype=torch.float64, device=dev).reshape(5, 19)
    out["gathered"] = D.gather_frames(rows, 5).cpu().numpy()
    out["rows"] = rows.cpu().numpy()
    out["max"] = D.max_over_ranks(3.25, dev)
    t = torch.full((1024,), 2.0, device=dev)
    dist.all_reduce(t)
    out["allreduce"] = t.cpu().numpy()
    dist.barrier()
    sd = synthetic.make_state_dict(0)
    n1, n3 = 512, 2048
    data, _, _ = synthetic.make_matcher_inputs(n1, n3, 8, seed=3, batch=1)
    m = matcher.from_state_dict(sd)
    sm = ShardedMatcher(m, data["keypoints3d"][0], data["descriptors3d_db"][0],
                        data["descriptors2d_db"][0], n1, dev)
    calls = []
    cb = sm._allgather
    sm._cb = None

    def counting(nbytes, stream, user):
        calls.append(int(nbytes))
        return cb(nbytes, stream, user)
    from onepose_amd import _lib
    sm._cb = _lib.ALLGATHER_FN(counting)
    d2 = torch.from_numpy(data["descriptors2d_query"]).to(dev)
    m0, m1, s0, s1 = sm.match(d2)
    torch.cuda.synchronize()
    out.update(m0=m0.cpu().numpy(), m1=m1.cpu().numpy(), s0=s0.cpu().numpy(),
               s1=s1.cpu().numpy(), ncalls=len(calls))
    inp = {k: torch.from_numpy(v).to(dev) for k, v in data.items()}
    pred, _ = m(inp)
    out.update(w0=pred["matches0"].cpu().numpy(), w1=pred["matches1"].cpu().numpy(),
               ws0=pred["matching_scores0"].cpu().numpy(),
               ws1=pred["matching_scores1"].cpu().numpy())
    np.savez(os.path.join(out_dir, "rccl.npz"), **out)
    dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_rccl_world1_collectives_and_sharded_matcher(tmp_path):
    mp.start_processes(_worker, args=(_free_port(), str(tmp_path)), nprocs=1, join=True,
                       start_method="spawn")
    r = np.load(tmp_path / "rccl.npz")
    assert str(r["backend"]) == "nccl"
    np.testing.assert_array_equal(r["gathered"], r["rows"])
    assert float(r["max"]) == 3.25
    np.testing.assert_array_equal(r["allreduce"], np.full(1024, 2.0, np.float32))
    # 8 attention layers x (KV + InstanceNorm) + row stats + row winners + column winners
    assert int(r["ncalls"]) == 8 * 2 + 3
    assert_pred_equal({"matches0": r["m0"][0], "matches1": r["m1"][0],
                       "matching_scores0": r["s0"][0], "matching_scores1": r["s1"][0]},
                      {"matches0": r["w0"], "matches1": r["w1"], "matching_scores0": r["ws0"],
                       "matching_scores1": r["ws1"]}, "RCCL world 1 sharded vs whole")
    assert (r["w0"] > -1).sum() > 100
