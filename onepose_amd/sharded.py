"""N3-sharded single-frame matching (SURVEY.md §8e optional / §8f rank 4).

One object's 3D points are split over the ranks of a ``torch.distributed`` group (one
process per GPU); every rank keeps the whole 2D side.  ``onepose_match_sharded`` runs the
GATsSPG forward on the rank's shard and exchanges, per attention layer, the 3D side's KV /
sum phi(k) and InstanceNorm moments, and after the score GEMM the row softmax statistics and
the row / column winners -- each an all-gather of one small fixed-size block per rank (about
66 KB per layer at batch 1), merged in rank order on the device.  Every rank ends with the
whole frame's matches.  For clouds too large for one GPU's latency budget (config 3, 16k+
points); frame-parallel sharding (``onepose_amd.distributed``) stays the throughput path.

The all-gather is a ctypes callback into ``torch.distributed``: RCCL
(``all_gather_into_tensor`` on the current stream) or, on a gloo group, a synchronous
host round trip (tests run two ranks on one GPU that way)."""
from __future__ import annotations

import ctypes
import traceback

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from .matcher import GATsSuperGlue, _hp


def shard_range(n3_total: int, world: int, rank: int):
    """Rank `rank`'s points [start, start + count) (onepose_shard_range's rule)."""
    start = n3_total * rank // world
    return start, n3_total * (rank + 1) // world - start


class ShardedMatcher:
    def __init__(self, matcher: GATsSuperGlue, keypoints3d, desc3d, leaves, n1: int, device,
                 batch: int = 1, group=None):
        self.lib = _lib.load()
        self.dev = torch.device(device)
        self.group = group
        if dist.is_available() and dist.is_initialized():
            self.world, self.rank = dist.get_world_size(group), dist.get_rank(group)
            self.backend = dist.get_backend(group)
        else:
            self.world, self.rank, self.backend = 1, 0, None
        self.B, self.n1 = int(batch), int(n1)
        self.matcher = matcher
        self.precision = matcher.precision
        self.scale_factor = float(_hp(matcher.hparams, "scale_factor"))
        self.threshold = float(_hp(matcher.hparams, "match_threshold"))
        f32 = dict(dtype=torch.float32, device=self.dev)
        d3 = torch.as_tensor(np.asarray(desc3d), dtype=torch.float32).reshape(256, -1)
        lv = torch.as_tensor(np.asarray(leaves), dtype=torch.float32).reshape(256, -1)
        self.n3 = d3.shape[1]
        self.L = lv.shape[1] // self.n3
        self.start, self.count = shard_range(self.n3, self.world, self.rank)
        s, c, L = self.start, self.count, self.L
        self.desc3d = d3[:, s:s + c].contiguous().to(self.dev)
        shard_leaves = lv[:, s * L:(s + c) * L].contiguous().to(self.dev)
        self.leaves_pm = torch.empty(c * L * 256, **f32)
        _lib.check(self.lib.onepose_prepare_leaves(shard_leaves.data_ptr(), 0, 1, c, L,
                                                   self.leaves_pm.data_ptr(),
                                                   _lib.stream_ptr(self.dev)), "prepare_leaves")
        self.weights = matcher.packed_weights(self.dev)
        xb = self.lib.onepose_match_sharded_xchg_bytes(self.B, self.n1, self.n3, self.world)
        self.xchg_bytes = xb
        self.send = torch.empty(xb, dtype=torch.uint8, device=self.dev)
        self.recv = torch.empty(self.world * xb, dtype=torch.uint8, device=self.dev)
        wb = self.lib.onepose_match_sharded_workspace_bytes(self.B, self.n1, self.n3, self.world,
                                                            self.rank, L, 0)
        self.ws_bytes = wb
        self.ws = torch.empty(wb, dtype=torch.uint8, device=self.dev)
        B = self.B
        self.matches0 = torch.empty(B, n1, dtype=torch.int64, device=self.dev)
        self.matches1 = torch.empty(B, self.n3, dtype=torch.int64, device=self.dev)
        self.mscores0 = torch.empty(B, n1, **f32)
        self.mscores1 = torch.empty(B, self.n3, **f32)
        self._error = None
        self._cb = _lib.ALLGATHER_FN(self._allgather)   # keep a reference

    def _allgather(self, nbytes, stream, user):
        try:
            send = self.send[:nbytes]
            recv = self.recv[:self.world * nbytes]
            if self.backend == "nccl":   # RCCL, enqueued on the matcher's (current) stream
                dist.all_gather_into_tensor(recv, send, group=self.group)
            elif self.world == 1:
                recv.copy_(send)
            else:   # gloo: host round trip, ordered by synchronising the matcher's stream
                torch.cuda.current_stream(self.dev).synchronize()
                cpu = send.cpu()
                outs = [torch.empty_like(cpu) for _ in range(self.world)]
                dist.all_gather(outs, cpu, group=self.group)
                recv.copy_(torch.cat(outs))
            return 0
        except Exception:   # reported through onepose_last_error's status
            self._error = traceback.format_exc()
            return 1

    def match(self, desc2d):
        """desc2d [B, 256, n1] on this rank's GPU -> (matches0 [B,n1], matches1 [B,n3],
        mscores0, mscores1), the whole frame's results on every rank."""
        d2 = desc2d.float().contiguous()
        assert tuple(d2.shape) == (self.B, 256, self.n1), tuple(d2.shape)
        rc = self.lib.onepose_match_sharded(
            self.weights.data_ptr(), d2.data_ptr(), 256 * self.n1, self.desc3d.data_ptr(), 0,
            self.leaves_pm.data_ptr(), 0, self.B, self.n1, self.n3, self.L, self.world,
            self.rank, self.scale_factor, self.threshold, self.precision,
            self.send.data_ptr(), self.recv.data_ptr(), self.xchg_bytes, self._cb, None,
            self.matches0.data_ptr(), self.matches1.data_ptr(), self.mscores0.data_ptr(),
            self.mscores1.data_ptr(), None, self.ws.data_ptr(), self.ws_bytes,
            _lib.stream_ptr(self.dev))
        if rc != 0 and self._error:
            raise RuntimeError(f"onepose_match_sharded: all-gather failed\n{self._error}")
        _lib.check(rc, "onepose_match_sharded")
        return self.matches0, self.matches1, self.mscores0, self.mscores1
