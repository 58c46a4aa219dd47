"""Every buffer of a C-ABI forward -- packed weights, descriptors, outputs, workspace and, for
the cached forward, the object cache, its prepare workspace and the leaf table -- placed inside
an allocation whose guard bytes (256 KiB each side) hold 0x00, 0xFF (NaN) or 0x7F (3.4e38):
the outputs are bit-identical across the fills and no guard byte changes.  A kernel reading past
a buffer's edge (where another forward's nearly equal values may lie) or writing past it would
show here; `tests/test_matcher_gpu.py` poisons the workspace's own bytes."""
import numpy as np
import pytest
import torch

from onepose_amd import _lib, matcher, synthetic

pytestmark = pytest.mark.gpu

GUARD = 1 << 18


class _Guarded:
    def __init__(self, dev, fill):
        self.dev, self.fill, self.bufs = dev, fill, []

    def place(self, src):
        nb = src.numel() * src.element_size()
        big = torch.full((2 * GUARD + nb,), self.fill, dtype=torch.uint8, device=self.dev)
        view = big[GUARD:GUARD + nb].view(src.dtype).view(src.shape)
        view.copy_(src)
        self.bufs.append((big, nb))
        return view

    def empty(self, shape, dtype):
        return self.place(torch.zeros(shape, dtype=dtype, device=self.dev))

    def changed_guard_bytes(self):
        return sum(int((torch.cat([b[:GUARD], b[GUARD + nb:]]) != self.fill).sum())
                   for b, nb in self.bufs)


def _forward(m, lib, t, cached, fill, dev):
    g = _Guarded(dev, fill)
    d2, s2 = m._operand(t["descriptors2d_query"])
    d3, s3 = m._operand(t["descriptors3d_db"])
    db, sl = m._operand(t["descriptors2d_db"])
    B, n1, n3 = d2.shape[0], d2.shape[2], d3.shape[2]
    L = db.shape[2] // n3
    w = g.place(m.packed_weights(dev))
    d2, d3, db = g.place(d2.contiguous()), g.place(d3.contiguous()), g.place(db.contiguous())
    m0, m1 = g.empty((B, n1), torch.int64), g.empty((B, n3), torch.int64)
    ms0, ms1 = g.empty((B, n1), torch.float32), g.empty((B, n3), torch.float32)
    conf = g.empty((B, n1, n3), torch.float32)
    wsb = _lib.workspace_bytes(lib, B, n1, n3, L, True, m.precision)
    ws = g.empty((wsb,), torch.uint8)
    sc, th = float(m.hparams["scale_factor"]), float(m.hparams["match_threshold"])
    s = _lib.stream_ptr(dev)
    if cached:
        pm = g.empty((n3 * L * 256,), torch.float32)
        _lib.check(lib.onepose_prepare_leaves_dt(db.data_ptr(), _lib.DT_F32, 0, 1, n3, L,
                                                 pm.data_ptr(), s), "leaves")
        cache = g.empty((_lib.object_cache_bytes(lib, n3, L, 0, m.precision) // 4,),
                        torch.float32)
        pwb = lib.onepose_object_prepare_workspace_bytes(n3, L)
        pws = g.empty((pwb,), torch.uint8)
        _lib.check(lib.onepose_object_prepare_dt(w.data_ptr(), d3.data_ptr(), _lib.DT_F32,
                                                 pm.data_ptr(), n3, L, m.precision, 0,
                                                 cache.data_ptr(), pws.data_ptr(), pwb, s),
                   "object_prepare")
        rc = lib.onepose_match_cached_dt(
            w.data_ptr(), d2.data_ptr(), _lib.DT_F32, s2, cache.data_ptr(), pm.data_ptr(), 0,
            B, n1, n3, L, sc, th, m.precision, 0, m0.data_ptr(), m1.data_ptr(), ms0.data_ptr(),
            ms1.data_ptr(), conf.data_ptr(), ws.data_ptr(), wsb, s)
        torch.cuda.synchronize()
        lib.onepose_object_release(cache.data_ptr())
        _lib.check(rc, "onepose_match_cached")
    else:
        _lib.check(lib.onepose_match_dt(
            w.data_ptr(), d2.data_ptr(), s2, d3.data_ptr(), s3, db.data_ptr(), sl, _lib.DT_F32,
            B, n1, n3, L, sc, th, m.precision, m0.data_ptr(), m1.data_ptr(), ms0.data_ptr(),
            ms1.data_ptr(), conf.data_ptr(), ws.data_ptr(), wsb, s), "onepose_match")
    torch.cuda.synchronize()
    return [x.cpu().numpy() for x in (m0, m1, ms0, ms1, conf)], g.changed_guard_bytes()


@pytest.mark.parametrize("precision", ["fp32", "fp32_split", "bf16"])
def test_forward_stays_inside_its_buffers(precision, device):
    lib = _lib.load()
    sd = synthetic.make_state_dict(3)
    data, _, _ = synthetic.make_matcher_inputs(300, 1000, 8, seed=9)   # ragged tiles both sides
    t = {k: torch.from_numpy(v).to(device) for k, v in data.items()}
    m = matcher.from_state_dict(sd, {**synthetic.DEFAULT_HPARAMS,
                                     "attention_precision": precision}).to(device)
    names = ("matches0", "matches1", "scores0", "scores1", "conf")
    for cached in (False, True):
        ref, changed = _forward(m, lib, t, cached, 0, device)
        assert changed == 0, f"cached={cached}: {changed} guard bytes written"
        for fill in (0xFF, 0x7F):
            out, changed = _forward(m, lib, t, cached, fill, device)
            assert changed == 0, f"cached={cached}, fill {fill:#x}: {changed} guard bytes written"
            for n, x, y in zip(names, ref, out):
                assert np.array_equal(x, y), f"cached={cached}: {n} depends on guard fill {fill:#x}"
