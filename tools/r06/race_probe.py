"""Round 6: do two matcher forwards running concurrently on two streams change each other's
bits?  (test_resident_object_forward's side-stream case read matching scores 1e-9 apart once.)

For each precision: a reference forward alone, then R rounds of the same forward on a side
stream while another forward runs on the default stream -- cached (resident object) and
uncached -- each compared bit for bit with the reference.  Prints the mismatch counts.
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from onepose_amd import matcher, synthetic  # noqa: E402


def run(precision, rounds=12, n1=300, n3=1000):
    dev = torch.device("cuda", 0)
    sd = synthetic.make_state_dict(3)
    hp = {**synthetic.DEFAULT_HPARAMS, "attention_precision": precision}
    res = matcher.from_state_dict(sd, hp).to(dev)
    unc = matcher.from_state_dict(sd, hp).to(dev)
    unc.resident_object = False
    data, _, _ = synthetic.make_matcher_inputs(n1, n3, 8, seed=9)
    t = {k: torch.from_numpy(v).to(dev) for k, v in data.items()}
    with torch.no_grad():
        ref, cref = unc(t)
        torch.cuda.synchronize()
        ref = {k: v.cpu().numpy() for k, v in ref.items()}
        cref = cref.cpu().numpy()
        res(t)
        torch.cuda.synchronize()
        side = torch.cuda.Stream(dev)
        bad = {"alone": 0, "cached side || uncached": 0, "uncached side || uncached": 0}

        def cmp(p, c):
            return int(any((p[k].cpu().numpy() != ref[k]).any() for k in ref)
                       or (c.cpu().numpy() != cref).any())

        for _ in range(rounds):
            p, c = res(t)
            torch.cuda.synchronize()
            bad["alone"] += cmp(p, c)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                ps, cs = res(t)
            pu, cu = unc(t)
            torch.cuda.synchronize()
            bad["cached side || uncached"] += cmp(ps, cs) + cmp(pu, cu)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                ps, cs = unc(t)
            pu, cu = unc(t)
            torch.cuda.synchronize()
            bad["uncached side || uncached"] += cmp(ps, cs) + cmp(pu, cu)
        # the test's sequence: a fresh prepare on the default stream, at once a cached forward
        # on the side stream (it waits for the prepare's event), then an uncached one
        bad["re-prepare, side || uncached"] = 0
        for _ in range(rounds):
            res._release_resident()
            res(t)
            with torch.cuda.stream(side):
                ps, cs = res(t)
            pu, cu = unc(t)
            torch.cuda.synchronize()
            bad["re-prepare, side || uncached"] += cmp(ps, cs) + cmp(pu, cu)
    print(precision, "mismatching forwards of", rounds, "/", 2 * rounds, "/", 2 * rounds, "/",
          2 * rounds, ":", bad, flush=True)
    return bad




def repeat_test(n=int(os.environ.get("RACE_N", "10"))):
    """test_resident_object_forward's whole body n times per precision in this process
    (RACE_PRECS="fp32_split" etc. to restrict)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
    import test_matcher_gpu as T
    dev = torch.device("cuda", 0)
    cases = [("fp32_split", False), ("fp32", False), ("bf16", False), ("fp32", True)]
    want = os.environ.get("RACE_PRECS")
    for prec, half in [c for c in cases if not want or c[0] in want.split(",")]:
        fails = 0
        for _ in range(n):
            try:
                T.test_resident_object_forward(prec, half, dev)
            except AssertionError as e:
                fails += 1
                print(prec, half, "FAIL:", str(e).splitlines()[:8], flush=True)
        print(prec, half, "failures", fails, "of", n, flush=True)


def variants(n=int(os.environ.get("RACE_N", "30"))):
    """Narrow the side-stream mismatch: which concurrency matters (fp32_split)."""
    dev = torch.device("cuda", 0)
    sd = synthetic.make_state_dict(3)
    hp = {**synthetic.DEFAULT_HPARAMS, "attention_precision": "fp32_split"}
    res = matcher.from_state_dict(sd, hp).to(dev)
    unc = matcher.from_state_dict(sd, hp).to(dev)
    unc.resident_object = False
    data, _, _ = synthetic.make_matcher_inputs(300, 1000, 8, seed=9)
    t = {k: torch.from_numpy(v).to(dev) for k, v in data.items()}
    with torch.no_grad():
        ref, cref = unc(t)
        torch.cuda.synchronize()
        ref = {k: v.cpu().numpy() for k, v in ref.items()}
        cref = cref.cpu().numpy()

        def bad(p, c):
            return int(any((p[k].cpu().numpy() != ref[k]).any() for k in ref)
                       or (c.cpu().numpy() != cref).any())

        counts = {"V1 prepare synced, side alone": 0, "V2 side || prepare + forward": 0,
                  "V3 side || forward (no re-prepare)": 0, "V4 side || prepare, no forward": 0}
        for _ in range(n):
            side = torch.cuda.Stream(dev)
            res._release_resident()
            res(t)
            torch.cuda.synchronize()
            with torch.cuda.stream(side):
                p, c = res(t)
            torch.cuda.synchronize()
            counts["V1 prepare synced, side alone"] += bad(p, c)
            res._release_resident()
            res(t)
            with torch.cuda.stream(side):
                p, c = res(t)
            torch.cuda.synchronize()
            counts["V2 side || prepare + forward"] += bad(p, c)
            res(t)
            with torch.cuda.stream(side):
                p, c = res(t)
            torch.cuda.synchronize()
            counts["V3 side || forward (no re-prepare)"] += bad(p, c)
            res._release_resident()
            d3, _ = res._operand(t["descriptors3d_db"])
            db, _ = res._operand(t["descriptors2d_db"])
            res._resident(t["descriptors3d_db"], t["descriptors2d_db"], d3, db, d3.shape[2],
                          db.shape[2] // d3.shape[2], False, dev)
            with torch.cuda.stream(side):
                p, c = res(t)
            torch.cuda.synchronize()
            counts["V4 side || prepare, no forward"] += bad(p, c)
    print("fp32_split side-stream mismatches of", n, ":", counts, flush=True)


def stress(n=int(os.environ.get("RACE_N", "40")), prec=os.environ.get("RACE_PREC", "fp32_split")):
    """Uncached forwards on the default stream while several cached (or uncached) forwards run
    on a side stream; every default-stream result against the sequential reference."""
    dev = torch.device("cuda", 0)
    sd = synthetic.make_state_dict(3)
    hp = {**synthetic.DEFAULT_HPARAMS, "attention_precision": prec}
    res = matcher.from_state_dict(sd, hp).to(dev)
    unc = matcher.from_state_dict(sd, hp).to(dev)
    unc.resident_object = False
    unc2 = matcher.from_state_dict(sd, hp).to(dev)
    unc2.resident_object = False
    data, _, _ = synthetic.make_matcher_inputs(300, 1000, 8, seed=9)
    t = {k: torch.from_numpy(v).to(dev) for k, v in data.items()}
    side = torch.cuda.Stream(dev)
    with torch.no_grad():
        ref, cref = unc(t)
        res(t)
        torch.cuda.synchronize()
        ref = {k: v.cpu().numpy() for k, v in ref.items()}
        cref = cref.cpu().numpy()
        counts = {"unc || 4 cached": 0, "unc || 4 uncached": 0, "cached || 4 uncached": 0}
        for _ in range(n):
            for key, bg, fg in (("unc || 4 cached", res, unc), ("unc || 4 uncached", unc2, unc),
                                ("cached || 4 uncached", unc2, res)):
                side.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(side):
                    for _ in range(4):
                        bg(t)
                outs = [fg(t) for _ in range(3)]
                torch.cuda.synchronize()
                for p, c in outs:
                    if (any((p[k].cpu().numpy() != ref[k]).any() for k in ref)
                            or (c.cpu().numpy() != cref).any()):
                        counts[key] += 1
    print(prec, "mismatching default-stream forwards of", 3 * n, ":", counts, flush=True)


def stress_prepare(n=int(os.environ.get("RACE_N", "30")),
                   prec=os.environ.get("RACE_PREC", "fp32_split")):
    """The object prepare (GAT 0, self-attention 1's and cross-attention 1's 3D halves -- the
    work only an uncached forward repeats) on the default stream while uncached forwards run on
    a side stream; each cache against one prepared alone, by layout region (floats)."""
    from onepose_amd import _lib
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    sd = synthetic.make_state_dict(3)
    hp = {**synthetic.DEFAULT_HPARAMS, "attention_precision": prec}
    m = matcher.from_state_dict(sd, hp).to(dev)
    unc = matcher.from_state_dict(sd, hp).to(dev)
    unc.resident_object = False
    data, _, _ = synthetic.make_matcher_inputs(300, 1000, 8, seed=9)
    t = {k: torch.from_numpy(v).to(dev) for k, v in data.items()}
    d3, _ = m._operand(t["descriptors3d_db"])
    db, _ = m._operand(t["descriptors2d_db"])
    n3, L = d3.shape[2], db.shape[2] // d3.shape[2]
    w = m.packed_weights(dev)
    pm = torch.empty(n3 * L * 256, device=dev)
    _lib.check(lib.onepose_prepare_leaves_dt(db.data_ptr(), _lib.DT_F32, 0, 1, n3, L,
                                             pm.data_ptr(), _lib.stream_ptr(dev)), "leaves")
    nb = _lib.object_cache_bytes(lib, n3, L, 0, m.precision)
    wsb = lib.onepose_object_prepare_workspace_bytes(n3, L)

    def prepare():
        cache = torch.zeros(nb // 4, dtype=torch.float32, device=dev)
        ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
        _lib.check(lib.onepose_object_prepare_dt(w.data_ptr(), d3.data_ptr(), _lib.DT_F32,
                                                 pm.data_ptr(), n3, L, m.precision, 0,
                                                 cache.data_ptr(), ws.data_ptr(), wsb,
                                                 _lib.stream_ptr(dev)), "prepare")
        lib.onepose_object_release(cache.data_ptr())
        return cache

    ref = prepare()
    torch.cuda.synchronize()
    ref = ref.view(torch.int32).cpu().numpy()
    # region starts in floats (matcher.hip obj_layout, flags 0)
    kl = 16
    regions = {"state": 0, "logits": n3 * 256}
    regions["phiq"] = regions["logits"] + 3 * n3 * kl
    regions["acc"] = regions["phiq"] + n3 * 256
    regions["ksum"] = regions["acc"] + ((n3 + 63) // 64) * 64 * 512
    regions["mf+"] = regions["ksum"] + 256
    names = list(regions)
    hdr = nb // 4 - 16   # the header (64 B, its generation differs per prepare) excluded
    bad = {}
    side = torch.cuda.Stream(dev)
    alone = {}
    for _ in range(n):   # control: prepares alone
        c = prepare()
        torch.cuda.synchronize()
        k = int((c.view(torch.int32).cpu().numpy()[:hdr] != ref[:hdr]).sum())
        alone[k] = alone.get(k, 0) + 1
    print(prec, "lone prepares: differing element counts -> runs", alone, flush=True)
    with torch.no_grad():
        for _ in range(n):
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(4):
                    unc(t)
            c = prepare()
            torch.cuda.synchronize()
            diff = np.nonzero(c.view(torch.int32).cpu().numpy()[:hdr] != ref[:hdr])[0]
            for i in diff:
                r = max((k for k in names if regions[k] <= i), key=lambda k: regions[k])
                bad[r] = bad.get(r, 0) + 1
            if len(diff):
                bad["runs"] = bad.get("runs", 0) + 1
                bad.setdefault("per run", []).append(int(len(diff)))
    print(prec, "prepares under concurrency differing from the lone prepare, elements by region,",
          "of", n, "runs:", bad or "none", flush=True)


def stress_foreign(n=int(os.environ.get("RACE_N", "40")),
                   prec=os.environ.get("RACE_PREC", "fp32_split")):
    """Uncached forwards on the default stream while the side stream runs PyTorch's own kernels
    (fp32 GEMMs and a large copy) instead of matcher forwards."""
    dev = torch.device("cuda", 0)
    sd = synthetic.make_state_dict(3)
    hp = {**synthetic.DEFAULT_HPARAMS, "attention_precision": prec}
    unc = matcher.from_state_dict(sd, hp).to(dev)
    unc.resident_object = False
    data, _, _ = synthetic.make_matcher_inputs(300, 1000, 8, seed=9)
    t = {k: torch.from_numpy(v).to(dev) for k, v in data.items()}
    a = torch.randn(2048, 2048, device=dev)
    big = torch.empty(64 << 20, device=dev)
    side = torch.cuda.Stream(dev)
    with torch.no_grad():
        ref, cref = unc(t)
        torch.cuda.synchronize()
        ref = {k: v.cpu().numpy() for k, v in ref.items()}
        cref = cref.cpu().numpy()
        bad = 0
        for _ in range(n):
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(4):
                    a2 = a @ a
                    big.copy_(big.flip(0))
            outs = [unc(t) for _ in range(3)]
            torch.cuda.synchronize()
            for p, c in outs:
                if (any((p[k].cpu().numpy() != ref[k]).any() for k in ref)
                        or (c.cpu().numpy() != cref).any()):
                    bad += 1
        del a2
    print(prec, "uncached forwards beside PyTorch kernels differing from the lone forward:",
          bad, "of", 3 * n, flush=True)


def stress_bg(n=int(os.environ.get("RACE_N", "40")), prec=os.environ.get("RACE_PREC", "fp32_split"),
              bg_prec=os.environ.get("RACE_BG_PREC", "fp32")):
    """Uncached `prec` forwards on the default stream while cached forwards of another precision
    (`bg_prec`: different GEMM loops) run on the side stream."""
    dev = torch.device("cuda", 0)
    sd = synthetic.make_state_dict(3)
    unc = matcher.from_state_dict(sd, {**synthetic.DEFAULT_HPARAMS,
                                       "attention_precision": prec}).to(dev)
    unc.resident_object = False
    bg = matcher.from_state_dict(sd, {**synthetic.DEFAULT_HPARAMS,
                                      "attention_precision": bg_prec}).to(dev)
    data, _, _ = synthetic.make_matcher_inputs(300, 1000, 8, seed=9)
    t = {k: torch.from_numpy(v).to(dev) for k, v in data.items()}
    side = torch.cuda.Stream(dev)
    with torch.no_grad():
        ref, cref = unc(t)
        bg(t)
        torch.cuda.synchronize()
        ref = {k: v.cpu().numpy() for k, v in ref.items()}
        cref = cref.cpu().numpy()
        bad = 0
        for _ in range(n):
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(4):
                    bg(t)
            outs = [unc(t) for _ in range(3)]
            torch.cuda.synchronize()
            for p, c in outs:
                if (any((p[k].cpu().numpy() != ref[k]).any() for k in ref)
                        or (c.cpu().numpy() != cref).any()):
                    bad += 1
    print(prec, "uncached forwards beside cached", bg_prec, "forwards differing:", bad, "of",
          3 * n, flush=True)


def stress_stages(n=int(os.environ.get("RACE_N", "40")), prec=os.environ.get("RACE_PREC", "fp32_split")):
    """Uncached `prec` forwards on the default stream while the side stream re-runs one stage
    range of a cached split forward (onepose_match_cached_stages on a workspace a whole forward
    filled first): GNN layers only, or the tail only."""
    from onepose_amd import _lib
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    sd = synthetic.make_state_dict(3)
    hp = {**synthetic.DEFAULT_HPARAMS, "attention_precision": prec}
    unc = matcher.from_state_dict(sd, hp).to(dev)
    unc.resident_object = False
    bgm = matcher.from_state_dict(sd, hp).to(dev)
    data, _, _ = synthetic.make_matcher_inputs(300, 1000, 8, seed=9)
    t = {k: torch.from_numpy(v).to(dev) for k, v in data.items()}
    side = torch.cuda.Stream(dev)
    with torch.no_grad():
        ref, cref = unc(t)
        bgm(t)   # builds the object cache
        torch.cuda.synchronize()
        ref = {k: v.cpu().numpy() for k, v in ref.items()}
        cref = cref.cpu().numpy()
        obj = bgm._obj
        d2, s2 = bgm._operand(t["descriptors2d_query"])
        B, n1, n3, L = 1, 300, 1000, 8
        w = bgm.packed_weights(dev)
        m0 = torch.empty(B, n1, dtype=torch.int64, device=dev)
        m1 = torch.empty(B, n3, dtype=torch.int64, device=dev)
        ms0, ms1 = torch.empty(B, n1, device=dev), torch.empty(B, n3, device=dev)
        conf = torch.empty(B, n1, n3, device=dev)
        wsb = _lib.workspace_bytes(lib, B, n1, n3, L, True, bgm.precision)
        with torch.cuda.stream(side):
            ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
        sc, th = float(hp["scale_factor"]), float(hp["match_threshold"])

        def stages(first, last):
            _lib.check(lib.onepose_match_cached_stages(
                w.data_ptr(), d2.data_ptr(), _lib.DT_F32, s2, obj["cache"].data_ptr(),
                obj["pm"].data_ptr(), 0, B, n1, n3, L, sc, th, bgm.precision, 0, m0.data_ptr(),
                m1.data_ptr(), ms0.data_ptr(), ms1.data_ptr(), conf.data_ptr(), ws.data_ptr(), wsb,
                first, last, side.cuda_stream), "stages")

        side.wait_stream(torch.cuda.current_stream(dev))
        stages(_lib.STAGE_INPUTS, _lib.STAGE_WINNERS)
        torch.cuda.synchronize()
        for name, (a, b) in (("layers", (_lib.STAGE_LAYER0, _lib.STAGE_FINAL - 1)),
                             ("tail", (_lib.STAGE_FINAL, _lib.STAGE_WINNERS)),
                             ("whole", (_lib.STAGE_INPUTS, _lib.STAGE_WINNERS))):
            bad = 0
            for _ in range(n):
                side.wait_stream(torch.cuda.current_stream(dev))
                for _ in range(4):
                    stages(a, b)
                outs = [unc(t) for _ in range(3)]
                torch.cuda.synchronize()
                for p, c in outs:
                    if (any((p[k].cpu().numpy() != ref[k]).any() for k in ref)
                            or (c.cpu().numpy() != cref).any()):
                        bad += 1
            print(prec, "uncached forwards beside cached-forward stages", name, "differing:",
                  bad, "of", 3 * n, flush=True)


if __name__ == "__main__":
    if sys.argv[1:] == ["test"]:
        repeat_test()
    elif sys.argv[1:] == ["variants"]:
        variants()
    elif sys.argv[1:] == ["stress"]:
        stress()
    elif sys.argv[1:] == ["prepare"]:
        stress_prepare()
    elif sys.argv[1:] == ["foreign"]:
        stress_foreign()
    elif sys.argv[1:] == ["bg"]:
        stress_bg()
    elif sys.argv[1:] == ["stages"]:
        stress_stages()
    else:
        for prec in sys.argv[1:] or ["fp32", "fp32_split", "bf16"]:
            run(prec)
