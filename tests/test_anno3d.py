"""The 3D-annotation producer: onepose_amd.data_utils.mean_descriptors /
mean_scores / save_object_annotations against the reference's own feature_process functions
(feature_process.py:191-194, 297-317, 352-363), bit for bit, through the fixture
tests/golden/anno3d.npz (make_golden.py anno3d_case), and read back the way inference.py:113-130
reads an object."""
import hashlib
import os

import numpy as np
import pytest

from conftest import golden
from onepose_amd import data_utils


def sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


@pytest.mark.parametrize("tag", ["f32", "f64"])
def test_anno3d_producer_matches_reference(tmp_path, tag):
    g = golden("anno3d")
    pre = f"{tag}_anno_3d_"
    desc = np.ascontiguousarray(g[pre + "collect_descriptors3d"].T)   # [sum(idxs), 256]
    scores = g[pre + "collect_scores3d"]
    idxs = g[f"{tag}_idxs"]
    xyzs = g[pre + "collect_keypoints3d"]
    assert sha(desc, scores, idxs, xyzs) == str(g[f"{tag}_inputs_sha"])
    avg = data_utils.mean_descriptors(desc, idxs)
    ref = g[pre + "average_descriptors3d"].T
    assert avg.dtype == ref.dtype and avg.shape == ref.shape
    assert np.array_equal(avg, ref)              # the reference does not renormalise
    assert np.array_equal(data_utils.mean_scores(scores, idxs), g[pre + "average_scores3d"])
    d = str(tmp_path / "anno")
    data_utils.save_object_annotations(d, xyzs, desc.T, scores, idxs)
    for f in ("anno_3d_average", "anno_3d_collect"):
        z = np.load(os.path.join(d, f + ".npz"))
        keys = sorted(k[len(f"{tag}_{f}_"):] for k in g.files if k.startswith(f"{tag}_{f}_"))
        assert sorted(z.files) == keys
        for k in keys:
            r = g[f"{tag}_{f}_{k}"]
            assert z[k].dtype == r.dtype and np.array_equal(z[k], r), (f, k)
    ids = np.load(os.path.join(d, "idxs.npy"))
    assert ids.dtype == idxs.dtype and np.array_equal(ids, idxs)
    # read back as inference.py:113-130 does (num_3d from the collect file's keypoints)
    np.random.seed(12345)
    kp3, avg_t, leaves = data_utils.load_object_annotations(d, num_leaf=8)
    assert kp3.shape == (len(idxs), 3) and avg_t.shape == (256, len(idxs))
    assert leaves.shape == (256, 8 * len(idxs))
    np.testing.assert_array_equal(avg_t.numpy(), ref.T.astype(np.float32))
