"""Pin the SuperPoint oracle (oracle/superpoint_np.py) to the reference module's own outputs
(tests/golden/superpoint.npz: superpoint.py run on seeded weights and images in the build
container, extraction config of extract_features.py:19-24 -> nms_radius 3, threshold 0.005,
max_keypoints 4096 / 300)."""
import hashlib

import numpy as np
import pytest

from conftest import golden
from onepose_amd import synthetic
from oracle import superpoint_np as O

CASES = {"sq": (128, 128, 0, 4096), "topk": (96, 160, 1, 300)}


def case(tag):
    h, w, seed, max_kp = CASES[tag]
    sd = synthetic.superpoint_state_dict(seed)
    sha = hashlib.sha256()
    for k in sorted(sd):
        sha.update(np.ascontiguousarray(sd[k]).tobytes())
    g = golden("superpoint")
    assert sha.hexdigest() == str(g[f"{tag}_weights_sha"]), "weight generator drifted"
    return sd, synthetic.superpoint_image(h, w, seed), max_kp, g


@pytest.mark.parametrize("tag", sorted(CASES))
def test_dense_maps_match_reference(tag):
    sd, img, _, g = case(tag)
    x = O.encoder(sd, img)
    np.testing.assert_allclose(O.score_map(sd, x), g[f"{tag}_score_map"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(O.dense_descriptors(sd, x), g[f"{tag}_dense_desc"], atol=2e-5)


@pytest.mark.parametrize("tag", sorted(CASES))
def test_detector_tail_is_exact_on_reference_maps(tag):
    """NMS + threshold + borders + top-k + sampling from the reference's own score map and
    dense descriptors: keypoints and scores bit-exact, descriptors to float rounding."""
    _, _, max_kp, g = case(tag)
    kp, sc = O.select_keypoints(O.simple_nms(g[f"{tag}_score_map"], 3), 0.005, 4, max_kp)
    np.testing.assert_array_equal(kp, g[f"{tag}_keypoints"])
    np.testing.assert_array_equal(sc, g[f"{tag}_scores"])
    desc = O.sample_descriptors(kp[None], g[f"{tag}_dense_desc"][None], 8, False)[0]
    np.testing.assert_allclose(desc, g[f"{tag}_descriptors"], atol=1e-6)


@pytest.mark.parametrize("tag", sorted(CASES))
def test_full_forward_matches_reference(tag):
    sd, img, max_kp, g = case(tag)
    kp, sc, desc = O.forward(sd, img, nms_radius=3, keypoint_threshold=0.005, remove_borders=4,
                             max_keypoints=max_kp, align_corners=False)
    np.testing.assert_array_equal(kp, g[f"{tag}_keypoints"])
    np.testing.assert_allclose(sc, g[f"{tag}_scores"], rtol=1e-4)
    np.testing.assert_allclose(desc, g[f"{tag}_descriptors"], atol=2e-5)


def test_topk_case_exercises_truncation():
    g = golden("superpoint")
    kp_all, _ = O.select_keypoints(O.simple_nms(g["topk_score_map"], 3), 0.005, 4, -1)
    assert len(kp_all) > 300 and len(g["topk_keypoints"]) == 300
    s = g["topk_scores"]
    assert np.all(s[:-1] >= s[1:])


def test_simple_nms_keeps_plateau_and_isolated_maxima():
    s = np.zeros((16, 16), np.float32)
    s[5, 5] = 0.9
    s[5, 7] = 0.5          # inside 0.9's window: suppressed
    s[12, 12] = 0.3
    s[12, 13] = 0.3        # equal neighbours are both maxima of the first pass
    out = O.simple_nms(s, 2)
    assert out[5, 5] == np.float32(0.9) and out[5, 7] == 0
    assert out[12, 12] == np.float32(0.3) and out[12, 13] == np.float32(0.3)


@pytest.mark.parametrize("tag", sorted(CASES))
def test_torch_cpu_restatement_matches_reference(tag):
    """oracle/superpoint_torch.py (the PyTorch-CPU detector bench.py's e2e cpu_baseline
    times) against the reference's outputs: score map, and the keypoint set (torch.topk's
    order among equal scores is unspecified) with its scores and descriptors."""
    from oracle import superpoint_torch as ST
    sd, img, max_kp, g = case(tag)
    kp, sc, desc, smap = ST.forward(ST.to_torch(sd), img, nms_radius=3, keypoint_threshold=0.005,
                                    remove_borders=4, max_keypoints=max_kp)
    np.testing.assert_allclose(smap, g[f"{tag}_score_map"], rtol=1e-4, atol=1e-6)
    ref = g[f"{tag}_keypoints"]
    assert len(kp) == len(ref)
    key = lambda k: np.lexsort((k[:, 0], k[:, 1]))   # noqa: E731
    o, r = key(kp), key(ref)
    np.testing.assert_array_equal(kp[o], ref[r])
    np.testing.assert_allclose(sc[o], g[f"{tag}_scores"][r], rtol=1e-4)
    np.testing.assert_allclose(desc[:, o], g[f"{tag}_descriptors"][:, r], atol=2e-5)
