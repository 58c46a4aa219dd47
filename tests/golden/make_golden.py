"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Run here, in the build container, where /root/reference exists (it never exists on the GPU
box; the fixtures travel instead):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What is imported from the reference (read-only, nothing copied):
  * src.models.GATsSPG_architectures.GATs_SuperGlue.GATsSuperGlue  (torch only)
  * src.models.extractors.SuperPoint.superpoint.sample_descriptors (torch only)
  * src.models.extractors.SuperPoint.superpoint.SuperPoint           (torch only)
  * src.evaluators.cmd_evaluator.Evaluator                         (numpy only)
  * src.utils.data_utils.{pad_features3d_random, build_features3d_leaves} (numpy/torch; the
    module's unrelated top-level cv2 / loguru imports are satisfied by empty placeholder
    modules for the duration of the import only)
  * src.sfm.postprocess.feature_process.{mean_descriptors, mean_scores, save_3d_anno} (numpy;
    the module's top-level h5py import -- used only by functions not called here -- is
    satisfied the same way)

Inputs are regenerated from seeds by ``onepose_amd.synthetic`` (numpy RandomState), so
each fixture stores only outputs plus SHA-256 digests of the inputs and weights.
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)

from onepose_amd import synthetic  # noqa: E402


def sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def ref_matcher(sd, hparams):
    from src.models.GATsSPG_architectures.GATs_SuperGlue import GATsSuperGlue
    m = GATsSuperGlue(dict(hparams))
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return m.eval()


SAMPLE_COLS = 16


def matcher_case(name, n1, n3, L, batch, seed, well_conditioned, full_conf, per_layer):
    sd = synthetic.make_state_dict(seed, well_conditioned=well_conditioned)
    data, _, _ = synthetic.make_matcher_inputs(n1, n3, L, seed=seed, batch=batch)
    model = ref_matcher(sd, synthetic.DEFAULT_HPARAMS)
    tdata = {k: torch.from_numpy(v) for k, v in data.items()}
    calls = []
    hooks = []
    if per_layer:
        # record every layer's outputs in call order with forward hooks; the reference's
        # own AttentionalGNN.forward runs unmodified.
        for i, layer in enumerate(model.gnn.layers):
            hooks.append(layer.register_forward_hook(
                lambda mod, inp, out, i=i: calls.append((i, out.detach().clone()))))
    with torch.no_grad():
        pred, conf = model(tdata)
    for h in hooks:
        h.remove()
    layer_out = []
    if per_layer:
        d2, d3 = tdata["descriptors2d_query"].float(), tdata["descriptors3d_db"].float()
        it = iter(calls)
        for i, lname in enumerate(model.gnn.names):
            if lname == "GATs":
                _, o = next(it)
                d3 = o.permute(0, 2, 1)
            else:
                (_, a), (_, b) = next(it), next(it)
                d2, d3 = d2 + a, d3 + b          # GATs_SuperGlue.py:78,83
            layer_out.append((d2.numpy().copy(), d3.numpy().copy()))
    conf = conf.numpy()
    rs = np.random.RandomState(99)
    c2 = np.sort(rs.choice(n1, min(SAMPLE_COLS, n1), replace=False))
    c3 = np.sort(rs.choice(n3, min(SAMPLE_COLS, n3), replace=False))
    top2 = -np.sort(-conf, axis=2)[:, :, :2]
    top2c = -np.sort(-conf, axis=1)[:, :2, :]
    out = {
        "n1": n1, "n3": n3, "num_leaf": L, "batch": batch, "seed": seed,
        "well_conditioned": int(well_conditioned),
        "weights_sha": synthetic.state_dict_sha(sd),
        "inputs_sha": sha(*[data[k] for k in sorted(data)]),
        "matches0": pred["matches0"].numpy(), "matches1": pred["matches1"].numpy(),
        "matching_scores0": pred["matching_scores0"].numpy(),
        "matching_scores1": pred["matching_scores1"].numpy(),
        "row_top2": top2, "col_top2": top2c,
        "conf_row_sum": conf.sum(axis=2), "conf_col_sum": conf.sum(axis=1),
        "cols2d": c2, "cols3d": c3,
    }
    if full_conf:
        out["conf"] = conf
    if per_layer:
        out["layer_d2"] = np.stack([o[0][:, :, c2] for o in layer_out])   # [12,B,256,16]
        out["layer_d3"] = np.stack([o[1][:, :, c3] for o in layer_out])
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    nm = int((pred["matches0"].numpy() > -1).sum())
    print(f"{name}: N1={n1} N3={n3} L={L} B={batch} matches={nm}")


def matcher_c3_idx():
    """BASELINE config 3's shape (1024 x 16384, L = 8): the index + score golden of one frame,
    frame 0 of the batch tests/test_configs_gpu.py runs at B = 32."""
    matcher_case("matcher_c3_idx", 1024, 16384, 8, 1, 8, True, False, False)


def empty_case():
    sd = synthetic.make_state_dict(0)
    model = ref_matcher(sd, synthetic.DEFAULT_HPARAMS)
    data = {
        "keypoints2d": torch.zeros(1, 0, 2), "keypoints3d": torch.zeros(1, 5, 3),
        "descriptors2d_query": torch.zeros(1, 256, 0), "descriptors3d_db": torch.zeros(1, 256, 5),
        "descriptors2d_db": torch.zeros(1, 256, 40),
    }
    with torch.no_grad():
        out = model(data)
    assert isinstance(out, dict)
    np.savez_compressed(os.path.join(HERE, "matcher_empty.npz"),
                        matches0=out["matches0"].numpy(), matches1=out["matches1"].numpy(),
                        matching_scores0=out["matching_scores0"].numpy(),
                        matching_scores1=out["matching_scores1"].numpy(),
                        skip_train=int(out["skip_train"]))
    print("matcher_empty:", out["matches0"].dtype, out["matches1"].shape)


def sample_desc_case():
    from src.models.extractors.SuperPoint import superpoint as sp
    rs = np.random.RandomState(7)
    h = w = 64
    dense = rs.standard_normal((1, 256, h, w)).astype(np.float32)
    dense /= np.linalg.norm(dense, axis=1, keepdims=True)
    kp = rs.uniform(0, 512, size=(1, 300, 2)).astype(np.float32)
    kp[0, :8] = np.array([[0, 0], [511, 511], [0, 511], [511, 0], [3.5, 3.5], [4, 4],
                          [507.5, 12.25], [256, 256]], np.float32)   # borders / exact centres
    outs = {}
    torch_version = torch.__version__
    for ac in (True, False):
        # superpoint.py:108 picks align_corners from the torch version; force each branch.
        torch.__version__ = "1.8.0" if ac else "2.1.0"
        try:
            with torch.no_grad():
                o = sp.sample_descriptors(torch.from_numpy(kp), torch.from_numpy(dense), 8)
        finally:
            torch.__version__ = torch_version
        outs["out_align_true" if ac else "out_align_false"] = o.numpy()
    np.savez_compressed(os.path.join(HERE, "sample_descriptors.npz"), dense_sha=sha(dense),
                        kp_sha=sha(kp), **outs)
    print("sample_descriptors: ok")


def evaluator_case():
    from src.evaluators.cmd_evaluator import Evaluator
    rs = np.random.RandomState(11)
    preds, gts = [], []
    for i in range(40):
        R = synthetic.random_rotation(rs)
        t = np.array([0.0, 0.0, 0.4]) + rs.normal(0, 0.05, 3)
        gt = np.concatenate([R, t[:, None]], 1)
        ang = rs.uniform(0, 8) * np.pi / 180.0
        ax = rs.standard_normal(3); ax /= np.linalg.norm(ax)
        K = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
        dR = np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K
        dt = rs.normal(0, 0.03, 3)
        pred = np.concatenate([dR @ R, (t + dt)[:, None]], 1)
        if i % 5 == 0:
            pred = np.concatenate([pred, [[0, 0, 0, 1]]], 0)      # 4x4 input path
        preds.append(pred); gts.append(gt)
    ev = Evaluator()
    for p, g in zip(preds, gts):
        ev.evaluate(p, g)
    c1, c3, c5 = list(ev.cmd1), list(ev.cmd3), list(ev.cmd5)
    summ = ev.summarize()
    np.savez_compressed(os.path.join(HERE, "evaluator.npz"),
                        preds=np.array([p[:3] for p in preds]), pred_is44=np.array([p.shape[0] == 4 for p in preds]),
                        gts=np.array(gts), cmd1=np.array(c1), cmd3=np.array(c3), cmd5=np.array(c5),
                        summary=np.array([summ["cmd1"], summ["cmd3"], summ["cmd5"]]))
    print("evaluator:", summ)


def eval_record_case():
    """eval_utils.record_eval_result (eval_utils.py:7-15) on the Evaluator summary of
    evaluator_case's poses, written by the reference into a scratch directory; the file name
    and text are stored. eval_utils.py:1 imports cv2, which record_eval_result never uses."""
    import tempfile
    import types
    from src.evaluators.cmd_evaluator import Evaluator
    added = []
    if "cv2" not in sys.modules:
        sys.modules["cv2"] = types.ModuleType("cv2")
        added.append("cv2")
    try:
        from src.utils import eval_utils
    finally:
        for name in added:
            del sys.modules[name]
    z = np.load(os.path.join(HERE, "evaluator.npz"))
    ev = Evaluator()
    for p, g in zip(z["preds"], z["gts"]):
        ev.evaluate(p, g)
    summ = ev.summarize()
    with tempfile.TemporaryDirectory() as d:
        out_dir = os.path.join(d, "runs", "eval", "GATsSPG")
        eval_utils.record_eval_result(out_dir, "0408-colorbox-box", "colorbox-4", summ)
        names = os.listdir(out_dir)
        text = open(os.path.join(out_dir, names[0])).read()
    np.savez_compressed(os.path.join(HERE, "eval_record.npz"), names=np.array(names),
                        text=np.array(text), summary=np.array([summ["cmd1"], summ["cmd3"],
                                                               summ["cmd5"]]))
    print("eval_record:", names, repr(text))


def object_inputs(seed=21, n3=60, dim=256):
    """Synthetic SfM object: per-3D-point observation counts 1..12, unit descriptors."""
    rs = np.random.RandomState(seed)
    idxs = rs.randint(1, 13, size=n3).astype(np.int64)
    m = int(idxs.sum())
    desc = rs.randn(dim, m).astype(np.float32)
    desc /= np.linalg.norm(desc, axis=0, keepdims=True)
    scores = rs.rand(m, 1).astype(np.float32)
    avg = rs.randn(dim, n3).astype(np.float32)
    avg_scores = rs.rand(n3, 1).astype(np.float32)
    return idxs, desc, scores, avg, avg_scores


def object_case():
    """pad_features3d_random + build_features3d_leaves (data_utils.py:143-205) as
    inference.py:113-130 calls them after seed_everything(12345): padded and truncated
    targets, 8 and 3 leaves."""
    import types
    added = []
    for name in ("cv2", "loguru"):   # data_utils.py:1,5 import these; the two functions don't
        if name not in sys.modules:
            sys.modules[name] = types.ModuleType(name)
            added.append(name)
    if "loguru" in added:
        sys.modules["loguru"].logger = None
    try:
        from src.utils import data_utils as du
    finally:
        for name in added:
            del sys.modules[name]
    idxs, desc, scores, avg, avg_scores = object_inputs()
    out = {"inputs_sha": sha(idxs, desc, scores, avg, avg_scores)}
    for tag, n_target, num_leaf in (("pad8", 72, 8), ("trunc8", 50, 8), ("pad3", 64, 3)):
        np.random.seed(12345)
        a, a_s = du.pad_features3d_random(avg, avg_scores, n_target)
        leaves, l_s = du.build_features3d_leaves(desc, scores, idxs, n_target, num_leaf)
        out[f"{tag}_avg"] = a.numpy()
        out[f"{tag}_avg_scores"] = a_s.numpy()
        out[f"{tag}_leaves"] = leaves.numpy()
        out[f"{tag}_leaf_scores"] = l_s.numpy()
    np.savez_compressed(os.path.join(HERE, "object_leaves.npz"), **out)


def anno3d_case():
    """The 3D-annotation producer (feature_process.py:191-194, 297-317, 352-363): per-3D-point
    means of the observation descriptors / scores and the three files inference.py:113-115 reads,
    written by the reference's own save_3d_anno / np.save into a scratch directory and stored
    here as arrays (float32 descriptors as count_features reads them from the h5 features file,
    plus a float64 case)."""
    import tempfile
    import types
    added = []
    if "h5py" not in sys.modules:   # feature_process.py:1; the functions below never touch it
        sys.modules["h5py"] = types.ModuleType("h5py")
        added.append("h5py")
    try:
        from src.sfm.postprocess import feature_process as fp
    finally:
        for name in added:
            del sys.modules[name]
    out = {}
    rs = np.random.RandomState(31)
    for tag, n3, dtype in (("f32", 60, np.float32), ("f64", 24, np.float64)):
        idxs = rs.randint(1, 17, size=n3).astype(np.int64)   # track lengths
        m = int(idxs.sum())
        desc = rs.randn(m, 256).astype(dtype)                 # [sum(idxs), 256], gather order
        desc /= np.linalg.norm(desc, axis=1, keepdims=True)
        scores = rs.rand(m, 1).astype(dtype)
        xyzs = rs.uniform(-0.1, 0.1, (n3, 3))
        avg_d = fp.mean_descriptors(desc, idxs)
        avg_s = fp.mean_scores(scores, idxs)
        with tempfile.TemporaryDirectory() as d:
            fp.save_3d_anno(xyzs, avg_d, avg_s, os.path.join(d, "anno_3d_average.npz"))
            fp.save_3d_anno(xyzs, desc, scores, os.path.join(d, "anno_3d_collect.npz"))
            np.save(os.path.join(d, "idxs.npy"), idxs)                   # feature_process.py:362-363
            for f in ("anno_3d_average", "anno_3d_collect"):
                z = np.load(os.path.join(d, f + ".npz"))
                for k in z.files:
                    out[f"{tag}_{f}_{k}"] = z[k]
            out[f"{tag}_idxs"] = np.load(os.path.join(d, "idxs.npy"))
        # the inputs are the collect file's own arrays (descriptors3d = desc.T)
        out[f"{tag}_inputs_sha"] = sha(desc, scores, idxs, xyzs)
    np.savez_compressed(os.path.join(HERE, "anno3d.npz"), **out)
    print("anno3d: ok")


def superpoint_case():
    """SuperPoint.forward (superpoint.py:170-224) with the extraction config of
    extract_features.py:19-24 on seeded synthetic weights and images; also the dense score map
    (after softmax + pixel shuffle, before NMS) and the normalised dense descriptors, computed
    with the reference module's own layers in its forward order."""
    from src.models.extractors.SuperPoint.superpoint import SuperPoint
    out = {}
    for tag, h, w, seed, max_kp in (("sq", 128, 128, 0, 4096), ("topk", 96, 160, 1, 300)):
        conf = dict(synthetic.SUPERPOINT_CONF, max_keypoints=max_kp)
        m = SuperPoint(conf).eval()
        sd = synthetic.superpoint_state_dict(seed)
        m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        img = torch.from_numpy(synthetic.superpoint_image(h, w, seed))[None, None]
        with torch.no_grad():
            pred = m(img)
            r = torch.relu
            x = r(m.conv1b(r(m.conv1a(img))))
            x = m.pool(x)
            x = m.pool(r(m.conv2b(r(m.conv2a(x)))))
            x = m.pool(r(m.conv3b(r(m.conv3a(x)))))
            x = r(m.conv4b(r(m.conv4a(x))))
            sc = torch.nn.functional.softmax(m.convPb(r(m.convPa(x))), 1)[:, :-1]
            b, _, hc, wc = sc.shape
            sc = sc.permute(0, 2, 3, 1).reshape(b, hc, wc, 8, 8)
            sc = sc.permute(0, 1, 3, 2, 4).reshape(b, hc * 8, wc * 8)
            dd = torch.nn.functional.normalize(m.convDb(r(m.convDa(x))), p=2, dim=1)
        out[f"{tag}_keypoints"] = pred["keypoints"][0].numpy()
        out[f"{tag}_scores"] = pred["scores"][0].numpy()
        out[f"{tag}_descriptors"] = pred["descriptors"][0].numpy()
        out[f"{tag}_score_map"] = sc[0].numpy()
        out[f"{tag}_dense_desc"] = dd[0].numpy()
        out[f"{tag}_weights_sha"] = sha(*[sd[k] for k in sorted(sd)])
    np.savez_compressed(os.path.join(HERE, "superpoint.npz"), **out)


def main():
    assert os.path.isdir(REF), "the reference is only available in the build container"
    sys.path.insert(0, REF)
    torch.set_num_threads(8)
    only = sys.argv[1:]
    if only:   # e.g.  make_golden.py object_case
        for name in only:
            globals()[name]()
        return
    matcher_case("matcher_c1_wc", 256, 512, 8, 1, 0, True, True, True)
    matcher_case("matcher_c1_rand", 256, 512, 8, 1, 1, False, False, True)
    matcher_case("matcher_b2", 128, 192, 8, 2, 2, True, True, False)
    matcher_case("matcher_ragged", 100, 77, 3, 1, 3, True, True, True)
    matcher_case("matcher_c2_idx", 1024, 4096, 8, 1, 4, True, False, False)
    matcher_c3_idx()
    empty_case()
    sample_desc_case()
    evaluator_case()
    eval_record_case()
    object_case()
    superpoint_case()
    anno3d_case()


if __name__ == "__main__":
    main()
