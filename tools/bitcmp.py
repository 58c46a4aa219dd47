"""Bit-identity check of two library builds: the same matcher calls through each, outputs
compared bit for bit.  Each build runs in its own process (ONEPOSE_LIB selects the library):
    ONEPOSE_LIB=tools/ab/lib_base.so python tools/bitcmp.py dump /tmp/a.npz
    python tools/bitcmp.py dump /tmp/b.npz
    python tools/bitcmp.py cmp /tmp/a.npz /tmp/b.npz
Cases: the uncached forward (onepose_match_ex, conf) and the cached bench path
(onepose_object_prepare + onepose_match_cached, with and without GAT tables) in fp32, bf16 and
fp32_split, on ragged and batched shapes.  BITCMP_BIG=1 adds configs 5 and 3's shapes (2048 x
8192, 1024 x 16384: more than 64 score tiles per row); their conf matrices are compared by
SHA-256 digest."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

CASES = [(1024, 4096, 8, 1), (200, 777, 8, 2), (96, 300, 3, 1), (256, 1024, 12, 3)]
PRECS = ["fp32", "bf16", "fp32_split"]
if os.environ.get("BITCMP_BIG") == "1":
    CASES += [(2048, 8192, 8, 1), (1024, 16384, 8, 1)]


def _conf(c):
    x = c.cpu().numpy()
    if x.size > 8 << 20:   # (a digest: the bits, not the values, are compared)
        return np.frombuffer(hashlib.sha256(x.tobytes()).digest(), np.uint8).copy()
    return x


def dump(path):
    from onepose_amd import _lib, matcher, synthetic as S
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    out = {}
    for (n1, n3, L, B) in CASES:
        sd = S.make_state_dict(1)
        data, _, _ = S.make_matcher_inputs(n1, n3, L, seed=3, batch=B)
        t = {k: torch.from_numpy(v).to(dev) for k, v in data.items()}
        for pi, prec in enumerate(PRECS):
            m = matcher.from_state_dict(sd, {**S.DEFAULT_HPARAMS, "attention_precision": prec}).to(dev)
            with torch.no_grad():
                pred, conf = m(t)
            key = f"u_{n1}_{n3}_{L}_{B}_{prec}"
            for k, v in pred.items():
                out[f"{key}_{k}"] = v.cpu().numpy()
            out[f"{key}_conf"] = _conf(conf)
            # cached path (object = sample 0's object, all frames of the batch)
            w = m.packed_weights(dev)
            f32 = dict(dtype=torch.float32, device=dev)
            s = _lib.stream_ptr(dev)
            d3 = t["descriptors3d_db"][0].contiguous()
            lv = t["descriptors2d_db"][0].contiguous()
            pmv = torch.empty(lib.onepose_leaves_prepared_bytes(1, n3, L) // 4, **f32)
            _lib.check(lib.onepose_prepare_leaves(lv.data_ptr(), 0, 1, n3, L, pmv.data_ptr(), s), "lv")
            for flags in (0, _lib.OBJ_GAT_TABLES):
                cache = torch.empty(lib.onepose_object_cache_bytes(n3, L, flags) // 4, **f32)
                wsb = lib.onepose_object_prepare_workspace_bytes(n3, L)
                ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
                _lib.check(lib.onepose_object_prepare(w.data_ptr(), d3.data_ptr(), pmv.data_ptr(), n3,
                                                      L, pi, flags, cache.data_ptr(), ws.data_ptr(),
                                                      wsb, s), "prepare")
                d2 = t["descriptors2d_query"].contiguous()
                o = [torch.empty(B, n1, dtype=torch.int64, device=dev),
                     torch.empty(B, n3, dtype=torch.int64, device=dev),
                     torch.empty(B, n1, **f32), torch.empty(B, n3, **f32)]
                cf = torch.empty(B, n1, n3, **f32)
                wmb = lib.onepose_match_workspace_bytes(B, n1, n3, L, 1)
                wm = torch.empty(wmb, dtype=torch.uint8, device=dev)
                _lib.check(lib.onepose_match_cached(
                    w.data_ptr(), d2.data_ptr(), 256 * n1, cache.data_ptr(), pmv.data_ptr(), 0, B,
                    n1, n3, L, float(m.hparams["scale_factor"]), float(m.hparams["match_threshold"]),
                    pi, flags, *[x.data_ptr() for x in o], cf.data_ptr(), wm.data_ptr(), wmb, s),
                    "match_cached")
                torch.cuda.synchronize()
                lib.onepose_object_release(cache.data_ptr())
                ck = f"c{flags}_{n1}_{n3}_{L}_{B}_{prec}"
                for nm, x in zip(("m0", "m1", "s0", "s1"), o):
                    out[f"{ck}_{nm}"] = x.cpu().numpy()
                out[f"{ck}_conf"] = _conf(cf)
    np.savez(path, **out)
    print("dumped", len(out), "arrays to", path)


def cmp(a, b):
    A, Bz = np.load(a), np.load(b)
    bad = 0
    for k in sorted(A.files):
        x, y = A[k], Bz[k]
        same = x.shape == y.shape and np.array_equal(x.view(np.uint8), y.view(np.uint8))
        if not same:
            bad += 1
            d = np.abs(x.astype(np.float64) - y.astype(np.float64)).max() if x.shape == y.shape else None
            print("DIFF", k, x.shape, y.shape, "max|d|", d)
    print(f"{len(A.files) - bad} of {len(A.files)} arrays bit-identical")
    return bad == 0


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        sys.exit(0 if cmp(sys.argv[2], sys.argv[3]) else 1)
