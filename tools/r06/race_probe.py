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


if __name__ == "__main__":
    if sys.argv[1:] == ["test"]:
        repeat_test()
    elif sys.argv[1:] == ["variants"]:
        variants()
    else:
        for prec in sys.argv[1:] or ["fp32", "fp32_split", "bf16"]:
            run(prec)
