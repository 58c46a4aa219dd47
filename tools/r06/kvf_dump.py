"""Round 6: one config-2 forward per precision (uncached and cached) through the library named
by ONEPOSE_LIB, outputs saved to argv[1] (.npz) -- variant libraries compared bit for bit."""
import hashlib
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from onepose_amd import matcher, synthetic  # noqa: E402


def main(out):
    dev = torch.device("cuda", 0)
    sd = synthetic.make_state_dict(3)
    data, _, _ = synthetic.make_matcher_inputs(1024, 4096, 8, seed=5)
    t = {k: torch.from_numpy(v).to(dev) for k, v in data.items()}
    res = {}
    with torch.no_grad():
        for prec in ("fp32", "fp32_split", "bf16"):
            for cached in (False, True):
                m = matcher.from_state_dict(sd, {**synthetic.DEFAULT_HPARAMS,
                                                 "attention_precision": prec}).to(dev)
                m.resident_object = cached
                p, c = m(t)
                torch.cuda.synchronize()
                for k, v in p.items():
                    res[f"{prec}_{cached}_{k}"] = v.cpu().numpy()
                res[f"{prec}_{cached}_conf"] = np.frombuffer(   # (its digest: 16 MB each)
                    hashlib.sha256(c.cpu().numpy().tobytes()).digest(), np.uint8)
    np.savez(out, **res)
    print("saved", out, len(res), flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
