import numpy as np, torch, sys
sys.path.insert(0, '.')
from onepose_amd import matcher, synthetic
sd = synthetic.make_state_dict(11)
B = 16
data, _, _ = synthetic.make_matcher_inputs(1024, 4096, 4, seed=11, batch=B)
def run(d, expand):
    m = matcher.from_state_dict(sd, dict(synthetic.DEFAULT_HPARAMS)).to('cuda')
    t = {k: torch.from_numpy(v).cuda() for k, v in d.items()}
    if expand:
        for k in ("descriptors3d_db", "descriptors2d_db", "keypoints3d"):
            t[k] = t[k][:1].expand_as(t[k])
    with torch.no_grad():
        p, c = m(t)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in p.items()}, c.cpu().numpy()
p, c = run(data, True)
worst = 0
for b in (0, 7, 15):
    p1, c1 = run({k: v[b:b+1] for k, v in data.items()}, False)
    worst = max(worst, float(np.abs(c[b] - c1[0]).max()))
    if b == 0:
        print("match agree", (p["matches0"] == p1["matches0"]).mean(), (p["matches0"] > -1).sum())
print("max conf diff", worst)
assert worst < 2e-5
