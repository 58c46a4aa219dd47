"""Round 6: does any kernel of a forward read workspace it has not written in that forward?
The same forward (cached and uncached, each precision) on a workspace filled with zeros and on
one filled with a NaN byte pattern (0xFF); outputs must be bit-identical.  (A split-mode
forward on a side stream read matching scores 1e-9 apart, 1 time in 10:
tools/r06/race_probe.py test.)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from onepose_amd import _lib, matcher, synthetic  # noqa: E402


def forward(m, lib, t, cached, obj, fill, dev):
    """One forward of GATsSuperGlue `m` on inputs `t` through the C-ABI with a workspace whose
    bytes are all `fill` before the call."""
    d2, s2 = m._operand(t["descriptors2d_query"])
    d3, s3 = m._operand(t["descriptors3d_db"])
    db, sl = m._operand(t["descriptors2d_db"])
    B, n1, n3 = d2.shape[0], d2.shape[2], d3.shape[2]
    L = db.shape[2] // n3
    w = m.packed_weights(dev)
    m0 = torch.empty(B, n1, dtype=torch.int64, device=dev)
    m1 = torch.empty(B, n3, dtype=torch.int64, device=dev)
    ms0 = torch.empty(B, n1, device=dev)
    ms1 = torch.empty(B, n3, device=dev)
    conf = torch.empty(B, n1, n3, device=dev)
    wsb = _lib.workspace_bytes(lib, B, n1, n3, L, True, m.precision)
    ws = torch.full((wsb,), fill, dtype=torch.uint8, device=dev)
    sc, th = float(m.hparams["scale_factor"]), float(m.hparams["match_threshold"])
    s = _lib.stream_ptr(dev)
    if cached:
        _lib.check(lib.onepose_match_cached_dt(
            w.data_ptr(), d2.data_ptr(), _lib.DT_F32, s2, obj["cache"].data_ptr(),
            obj["pm"].data_ptr(), 0, B, n1, n3, L, sc, th, m.precision, 0, m0.data_ptr(),
            m1.data_ptr(), ms0.data_ptr(), ms1.data_ptr(), conf.data_ptr(), ws.data_ptr(), wsb,
            s), "cached")
    else:
        _lib.check(lib.onepose_match_dt(
            w.data_ptr(), d2.data_ptr(), s2, d3.data_ptr(), s3, db.data_ptr(), sl, _lib.DT_F32,
            B, n1, n3, L, sc, th, m.precision, m0.data_ptr(), m1.data_ptr(), ms0.data_ptr(),
            ms1.data_ptr(), conf.data_ptr(), ws.data_ptr(), wsb, s), "uncached")
    torch.cuda.synchronize()
    return [x.cpu().numpy() for x in (m0, m1, ms0, ms1, conf)]


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    sd = synthetic.make_state_dict(3)
    data, _, _ = synthetic.make_matcher_inputs(300, 1000, 8, seed=9)
    t = {k: torch.from_numpy(v).to(dev) for k, v in data.items()}
    for prec in ("fp32", "fp32_split", "bf16"):
        m = matcher.from_state_dict(sd, {**synthetic.DEFAULT_HPARAMS,
                                         "attention_precision": prec}).to(dev)
        d3, _ = m._operand(t["descriptors3d_db"])
        db, _ = m._operand(t["descriptors2d_db"])
        obj = m._resident(t["descriptors3d_db"], t["descriptors2d_db"], d3, db, d3.shape[2],
                          db.shape[2] // d3.shape[2], False, dev)
        torch.cuda.synchronize()
        for cached in (False, True):
            a = forward(m, lib, t, cached, obj, 0, dev)
            b = forward(m, lib, t, cached, obj, 255, dev)
            c = forward(m, lib, t, cached, obj, 0, dev)
            names = ("matches0", "matches1", "scores0", "scores1", "conf")
            diff = [n for n, x, y in zip(names, a, b) if not np.array_equal(x, y, equal_nan=True)]
            rep = [n for n, x, y in zip(names, a, c) if not np.array_equal(x, y, equal_nan=True)]
            print(f"{prec:10s} {'cached' if cached else 'uncached':8s} zero-vs-NaN workspace "
                  f"differs in {diff or 'nothing'}; zero-vs-zero in {rep or 'nothing'}",
                  flush=True)




def cache_poison():
    """The object cache: prepared into memory filled with zeros and with 0xFF bytes; the cached
    forwards on the two must be bit-identical (a region the prepare does not write but the
    forward reads would differ)."""
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    sd = synthetic.make_state_dict(3)
    data, _, _ = synthetic.make_matcher_inputs(300, 1000, 8, seed=9)
    t = {k: torch.from_numpy(v).to(dev) for k, v in data.items()}
    for prec in ("fp32", "fp32_split", "bf16"):
        m = matcher.from_state_dict(sd, {**synthetic.DEFAULT_HPARAMS,
                                         "attention_precision": prec}).to(dev)
        d3, _ = m._operand(t["descriptors3d_db"])
        db, _ = m._operand(t["descriptors2d_db"])
        n3, L = d3.shape[2], db.shape[2] // d3.shape[2]
        w = m.packed_weights(dev)
        pm = torch.empty(n3 * L * 256, device=dev)
        _lib.check(lib.onepose_prepare_leaves_dt(db.data_ptr(), _lib.DT_F32, 0, 1, n3, L,
                                                 pm.data_ptr(), _lib.stream_ptr(dev)), "leaves")
        outs = []
        for fill in (0, 255):   # the cache and the prepare's workspace both filled
            nb = _lib.object_cache_bytes(lib, n3, L, 0, m.precision)
            cache = torch.full((nb,), fill, dtype=torch.uint8, device=dev).view(torch.float32)
            wsb = lib.onepose_object_prepare_workspace_bytes(n3, L)
            ws = torch.full((wsb,), fill, dtype=torch.uint8, device=dev)
            _lib.check(lib.onepose_object_prepare_dt(w.data_ptr(), d3.data_ptr(), _lib.DT_F32,
                                                     pm.data_ptr(), n3, L, m.precision, 0,
                                                     cache.data_ptr(), ws.data_ptr(), wsb,
                                                     _lib.stream_ptr(dev)), "prepare")
            outs.append(forward(m, lib, t, True, {"cache": cache, "pm": pm}, 0, dev))
            lib.onepose_object_release(cache.data_ptr())
        names = ("matches0", "matches1", "scores0", "scores1", "conf")
        diff = [n for n, x, y in zip(names, outs[0], outs[1])
                if not np.array_equal(x, y, equal_nan=True)]
        print(f"{prec:10s} cache + prepare workspace on zeros vs 0xFF: differs in "
              f"{diff or 'nothing'}",
              flush=True)


if __name__ == "__main__":
    if sys.argv[1:] == ["cache"]:
        cache_poison()
    else:
        main()
