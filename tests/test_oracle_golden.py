"""Pin the numpy oracle (oracle/matcher_np.py) to fixtures produced by the reference itself
(tests/golden/make_golden.py, run in the build container)."""
import numpy as np
import pytest

from conftest import golden
from onepose_amd import synthetic
from oracle import matcher_np as M

CASES = ["matcher_c1_wc", "matcher_c1_rand", "matcher_b2", "matcher_ragged"]


def regen(g):
    n1, n3, L, B, seed, wc = [int(g[k]) for k in ("n1", "n3", "num_leaf", "batch", "seed",
                                                   "well_conditioned")]
    sd = synthetic.make_state_dict(seed, well_conditioned=bool(wc))
    assert synthetic.state_dict_sha(sd) == str(g["weights_sha"]), "weight generator drifted"
    data, obj, frames = synthetic.make_matcher_inputs(n1, n3, L, seed=seed, batch=B)
    return sd, data, frames


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference(name):
    g = golden(name)
    sd, data, _ = regen(g)
    import hashlib
    h = hashlib.sha256()
    for k in sorted(data):
        h.update(np.ascontiguousarray(data[k]).tobytes())
    assert h.hexdigest() == str(g["inputs_sha"]), "input generator drifted"
    rec = []
    pred, conf = M.forward(sd, data, record=rec)
    np.testing.assert_array_equal(pred["matches0"], g["matches0"])
    np.testing.assert_array_equal(pred["matches1"], g["matches1"])
    np.testing.assert_allclose(pred["matching_scores0"], g["matching_scores0"], atol=1e-5)
    np.testing.assert_allclose(pred["matching_scores1"], g["matching_scores1"], atol=1e-5)
    if "conf" in g:
        np.testing.assert_allclose(conf, g["conf"], atol=1e-5)
    np.testing.assert_allclose(conf.sum(axis=2), g["conf_row_sum"], rtol=1e-4, atol=1e-5)
    if "layer_d2" in g:
        for i in range(12):
            np.testing.assert_allclose(rec[i][0][:, :, g["cols2d"]], g["layer_d2"][i], atol=5e-5)
            np.testing.assert_allclose(rec[i][1][:, :, g["cols3d"]], g["layer_d3"][i], atol=5e-5)


def test_sample_descriptors_oracle():
    g = golden("sample_descriptors")
    rs = np.random.RandomState(7)
    dense = rs.standard_normal((1, 256, 64, 64)).astype(np.float32)
    dense /= np.linalg.norm(dense, axis=1, keepdims=True)
    kp = rs.uniform(0, 512, size=(1, 300, 2)).astype(np.float32)
    kp[0, :8] = np.array([[0, 0], [511, 511], [0, 511], [511, 0], [3.5, 3.5], [4, 4],
                          [507.5, 12.25], [256, 256]], np.float32)
    for ac in (True, False):
        out = M.sample_descriptors(kp, dense, 8, align_corners=ac)
        ref = g["out_align_true" if ac else "out_align_false"]
        np.testing.assert_allclose(out, ref, atol=2e-6)


def test_evaluator_matches_reference_fixture():
    from onepose_amd.pose import Evaluator, query_pose_error
    g = golden("evaluator")
    ev = Evaluator()
    for p, is44, gt in zip(g["preds"], g["pred_is44"], g["gts"]):
        if is44:
            p = np.concatenate([p, [[0, 0, 0, 1]]], 0)
        ev.evaluate(p, gt)
    np.testing.assert_array_equal(np.array(ev.cmd1), g["cmd1"])
    np.testing.assert_array_equal(np.array(ev.cmd3), g["cmd3"])
    np.testing.assert_array_equal(np.array(ev.cmd5), g["cmd5"])
    s = ev.summarize()
    np.testing.assert_allclose([s["cmd1"], s["cmd3"], s["cmd5"]], g["summary"])
    a, t = query_pose_error(g["preds"][1], g["gts"][1])
    assert np.isfinite(a) and np.isfinite(t)


def test_object_leaves_match_reference():
    """pad_features3d_random / build_features3d_leaves (data_utils.py:143-205), seeded as
    inference.py does (seed_everything(12345)): the reference's outputs, bit for bit."""
    import os
    import sys
    from conftest import REPO
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    from make_golden import object_inputs
    from onepose_amd import data_utils as DU
    g = golden("object_leaves")
    idxs, desc, scores, avg, avg_scores = object_inputs()
    for tag, n_target, num_leaf in (("pad8", 72, 8), ("trunc8", 50, 8), ("pad3", 64, 3)):
        np.random.seed(12345)
        a, a_s = DU.pad_features3d_random(avg, avg_scores, n_target)
        leaves, l_s = DU.build_features3d_leaves(desc, scores, idxs, n_target, num_leaf)
        np.testing.assert_array_equal(a.numpy(), g[f"{tag}_avg"])
        np.testing.assert_array_equal(a_s.numpy(), g[f"{tag}_avg_scores"])
        np.testing.assert_array_equal(leaves.numpy(), g[f"{tag}_leaves"])
        np.testing.assert_array_equal(l_s.numpy(), g[f"{tag}_leaf_scores"])


@pytest.mark.parametrize("name", CASES + ["matcher_c2_idx", "matcher_c3_idx"])
def test_torch_cpu_restatement_matches_reference(name):
    """oracle/matcher_torch.py (the PyTorch-CPU path bench.py's cpu_baseline times) against
    the reference's own outputs."""
    from oracle import matcher_torch as MT
    g = golden(name)
    sd, data, _ = regen(g)
    import hashlib
    h = hashlib.sha256()
    for k in sorted(data):
        h.update(np.ascontiguousarray(data[k]).tobytes())
    assert h.hexdigest() == str(g["inputs_sha"]), "input generator drifted"
    pred, conf = MT.forward(MT.to_torch(sd), data)
    np.testing.assert_array_equal(pred["matches0"], g["matches0"])
    np.testing.assert_array_equal(pred["matches1"], g["matches1"])
    np.testing.assert_allclose(pred["matching_scores0"], g["matching_scores0"], atol=1e-5)
    np.testing.assert_allclose(pred["matching_scores1"], g["matching_scores1"], atol=1e-5)
    if "conf" in g:
        np.testing.assert_allclose(conf, g["conf"], atol=1e-5)
    np.testing.assert_allclose(conf.sum(axis=2), g["conf_row_sum"], rtol=1e-4, atol=1e-5)
