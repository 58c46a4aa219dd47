"""Round 6: does any kernel of a forward read (or write) outside the buffers it is given?
Every buffer of one C-ABI forward -- packed weights, descriptors, outputs, workspace and, for the
cached forward, the object cache and leaf table -- is placed inside a larger allocation whose
guard bytes (1 MiB each side) are filled with 0x00, 0xFF (NaN) or 0x7F (3.4e38); the outputs
must be bit-identical across the fills, and the guards must keep their fill."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from onepose_amd import _lib, matcher, synthetic  # noqa: E402

GUARD = 1 << 20


class Guarded:
    def __init__(self, dev):
        self.dev, self.bufs = dev, []

    def place(self, src, fill):
        """A copy of `src` (contiguous) inside a guarded allocation."""
        nb = src.numel() * src.element_size()
        big = torch.full((2 * GUARD + nb,), fill, dtype=torch.uint8, device=self.dev)
        view = big[GUARD:GUARD + nb].view(src.dtype).view(src.shape)
        view.copy_(src)
        self.bufs.append((big, nb, fill))
        return view

    def empty(self, shape, dtype, fill):
        return self.place(torch.zeros(shape, dtype=dtype, device=self.dev), fill)

    def guards_intact(self):
        bad = 0
        for big, nb, fill in self.bufs:
            g = torch.cat([big[:GUARD], big[GUARD + nb:]])
            bad += int((g != fill).sum())
        return bad


def forward(m, lib, t, cached, fill, dev):
    g = Guarded(dev)
    d2, s2 = m._operand(t["descriptors2d_query"])
    d3, s3 = m._operand(t["descriptors3d_db"])
    db, sl = m._operand(t["descriptors2d_db"])
    for x in (d2, d3, db):
        assert x.is_contiguous()
    B, n1, n3 = d2.shape[0], d2.shape[2], d3.shape[2]
    L = db.shape[2] // n3
    w = g.place(m.packed_weights(dev), fill)
    d2, d3, db = g.place(d2, fill), g.place(d3, fill), g.place(db, fill)
    m0 = g.empty((B, n1), torch.int64, fill)
    m1 = g.empty((B, n3), torch.int64, fill)
    ms0 = g.empty((B, n1), torch.float32, fill)
    ms1 = g.empty((B, n3), torch.float32, fill)
    conf = g.empty((B, n1, n3), torch.float32, fill)
    wsb = _lib.workspace_bytes(lib, B, n1, n3, L, True, m.precision)
    ws = g.empty((wsb,), torch.uint8, fill)
    sc, th = float(m.hparams["scale_factor"]), float(m.hparams["match_threshold"])
    s = _lib.stream_ptr(dev)
    if cached:
        pm = g.empty((n3 * L * 256,), torch.float32, fill)
        _lib.check(lib.onepose_prepare_leaves_dt(db.data_ptr(), _lib.DT_F32, 0, 1, n3, L,
                                                 pm.data_ptr(), s), "leaves")
        nb = _lib.object_cache_bytes(lib, n3, L, 0, m.precision)
        cache = g.empty((nb // 4,), torch.float32, fill)
        pwb = lib.onepose_object_prepare_workspace_bytes(n3, L)
        pws = g.empty((pwb,), torch.uint8, fill)
        _lib.check(lib.onepose_object_prepare_dt(w.data_ptr(), d3.data_ptr(), _lib.DT_F32,
                                                 pm.data_ptr(), n3, L, m.precision, 0,
                                                 cache.data_ptr(), pws.data_ptr(), pwb, s),
                   "prepare")
        _lib.check(lib.onepose_match_cached_dt(
            w.data_ptr(), d2.data_ptr(), _lib.DT_F32, s2, cache.data_ptr(), pm.data_ptr(), 0,
            B, n1, n3, L, sc, th, m.precision, 0, m0.data_ptr(), m1.data_ptr(), ms0.data_ptr(),
            ms1.data_ptr(), conf.data_ptr(), ws.data_ptr(), wsb, s), "cached")
        torch.cuda.synchronize()
        lib.onepose_object_release(cache.data_ptr())
    else:
        _lib.check(lib.onepose_match_dt(
            w.data_ptr(), d2.data_ptr(), s2, d3.data_ptr(), s3, db.data_ptr(), sl, _lib.DT_F32,
            B, n1, n3, L, sc, th, m.precision, m0.data_ptr(), m1.data_ptr(), ms0.data_ptr(),
            ms1.data_ptr(), conf.data_ptr(), ws.data_ptr(), wsb, s), "uncached")
    torch.cuda.synchronize()
    return [x.cpu().numpy() for x in (m0, m1, ms0, ms1, conf)], g.guards_intact()


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    sd = synthetic.make_state_dict(3)
    names = ("matches0", "matches1", "scores0", "scores1", "conf")
    for n1, n3 in ((300, 1000), (1024, 4096)):
        data, _, _ = synthetic.make_matcher_inputs(n1, n3, 8, seed=9)
        t = {k: torch.from_numpy(v).to(dev) for k, v in data.items()}
        for prec in ("fp32", "fp32_split", "bf16"):
            m = matcher.from_state_dict(sd, {**synthetic.DEFAULT_HPARAMS,
                                             "attention_precision": prec}).to(dev)
            for cached in (False, True):
                outs = {f: forward(m, lib, t, cached, f, dev) for f in (0, 255, 127)}
                ref = outs[0][0]
                diff = {f: [n for n, x, y in zip(names, ref, o[0])
                            if not np.array_equal(x, y, equal_nan=True)]
                        for f, o in outs.items() if f != 0}
                print(f"{n1}x{n3} {prec:10s} {'cached' if cached else 'uncached':8s} "
                      f"outputs vs 0x00 guards: 0xFF {diff[255] or 'same'}, 0x7F "
                      f"{diff[127] or 'same'}; guard bytes changed: "
                      f"{[o[1] for o in outs.values()]}", flush=True)


if __name__ == "__main__":
    main()
