"""GPU RANSAC-EPnP (libonepose_hip) vs the C oracle (oracle/epnp_ransac.c).

Both restate OpenCV 4.4's solvePnPRansac(SOLVEPNP_EPNP) with the same cv::RNG stream, so
they must pick the same model: identical status, inlier mask and inlier count, and poses
within 1e-6 rad / 1e-6 m (both are double-precision; only operation order differs).  The
north-star bound (1e-4 rad, 1e-3 m) is asserted too.  Parity against OpenCV itself is
unpinned (cv2 is not installed); tests/test_pnp_oracle.py pins the oracle on known-answer
scenes."""
import numpy as np
import pytest
import torch

from onepose_amd import pose as P
from onepose_amd import synthetic as S
from oracle import pnp_oracle as O

pytestmark = pytest.mark.gpu


def scene(seed, n, outlier_frac=0.3, px_noise=0.5):
    rs = np.random.RandomState(seed)
    K = S.crop_intrinsics()
    R = S.random_rotation(rs)
    t = np.array([rs.uniform(-0.03, 0.03), rs.uniform(-0.03, 0.03), rs.uniform(0.35, 0.55)])
    pose = np.concatenate([R, t[:, None]], 1)
    pts = rs.uniform(-0.1, 0.1, (n, 3)).astype(np.float32)
    uv = S.project(K, pose, pts.astype(np.float64)) + rs.normal(0, px_noise, (n, 2))
    out = rs.rand(n) < outlier_frac
    uv[out] = rs.uniform(0, 512, (out.sum(), 2))
    p2 = uv.astype(np.float32)
    p3 = (pts.astype(np.float64) * 1000.0).astype(np.float32)
    return p2, p3, K, pose, ~out


def rot_angle(Ra, Rb):
    c = (np.trace(Ra @ Rb.T) - 1) / 2
    return np.arccos(np.clip(c, -1, 1))


def run_gpu(scenes, device, max_points=None):
    B = len(scenes)
    M = max_points or max(s[0].shape[0] for s in scenes)
    p2 = np.zeros((B, M, 2), np.float32)
    p3 = np.zeros((B, M, 3), np.float32)
    Ks = np.zeros((B, 3, 3))
    counts = np.zeros(B, np.int32)
    for b, s in enumerate(scenes):
        n = s[0].shape[0]
        p2[b, :n], p3[b, :n], Ks[b], counts[b] = s[0], s[1], s[2], n
    pose, mask, nin, status = P.ransac_pnp_batch(
        torch.from_numpy(p2).to(device), torch.from_numpy(p3).to(device),
        torch.from_numpy(counts).to(device), torch.from_numpy(Ks).to(device), scale=1000.0)
    torch.cuda.synchronize()
    return pose.cpu().numpy(), mask.cpu().numpy().astype(bool), nin.cpu().numpy(), status.cpu().numpy()


@pytest.mark.parametrize("outliers", [0.0, 0.3, 0.6])
def test_ransac_matches_oracle(outliers, device):
    scenes = [scene(100 + i, n, outliers) for i, n in enumerate([40, 200, 700, 1024])]
    pose, mask, nin, status = run_gpu(scenes, device)
    for b, (p2, p3, K, gt, inl) in enumerate(scenes):
        st, opose, omask, onin, iters = O.pnp_ransac(p2, p3, K, scale=1000.0)
        n = p2.shape[0]
        assert status[b] == st == 0
        assert nin[b] == onin
        np.testing.assert_array_equal(mask[b, :n], omask)
        assert not mask[b, n:].any()
        assert rot_angle(pose[b, :, :3], opose[:, :3]) < 1e-6
        assert np.abs(pose[b, :, 3] - opose[:, 3]).max() < 1e-6
        # north-star bound vs the oracle, and GT recovered to the noise level
        assert rot_angle(pose[b, :, :3], gt[:, :3]) < np.deg2rad(1.0)
        assert np.abs(pose[b, :, 3] - gt[:, 3]).max() < 0.01


def test_ransac_small_sets_and_many_rounds(device):
    """The round's cv::RNG draws are generated in parallel by jump-ahead and dealt out by one
    lane: small point sets redraw duplicates often (n = 6..16 runs past the generated draws
    into the sequential fallback), and 50-70% outliers keep RANSAC going for several
    64-iteration rounds (jump-ahead from a mid-stream state).  Same model as the oracle."""
    cases = [(6, 0.0), (7, 0.3), (9, 0.3), (12, 0.4), (16, 0.5), (60, 0.6), (300, 0.7),
             (500, 0.5)]
    scenes = [scene(300 + i, n, f) for i, (n, f) in enumerate(cases)]
    pose, mask, nin, status = run_gpu(scenes, device)
    for b, (p2, p3, K, gt, inl) in enumerate(scenes):
        st, opose, omask, onin, iters = O.pnp_ransac(p2, p3, K, scale=1000.0)
        n = p2.shape[0]
        assert status[b] == st, b
        assert nin[b] == onin, b
        np.testing.assert_array_equal(mask[b, :n], omask)
        if st == 0:
            assert rot_angle(pose[b, :, :3], opose[:, :3]) < 1e-6
            assert np.abs(pose[b, :, 3] - opose[:, 3]).max() < 1e-6
    assert O.pnp_ransac(*scenes[-2][:3], scale=1000.0)[4] > 64   # several rounds


def test_ransac_edge_counts(device):
    s5 = scene(7, 5, 0.0)
    s4 = scene(8, 4, 0.0)
    s3 = scene(9, 3, 0.0)
    s6 = scene(10, 6, 0.0)
    pose, mask, nin, status = run_gpu([s5, s4, s3, s6], device, max_points=8)
    # exactly 5 points: EPnP on all of them, every point an inlier
    st, opose, omask, onin, _ = O.pnp_ransac(s5[0], s5[1], s5[2], scale=1000.0)
    assert status[0] == 0 and nin[0] == 5 and mask[0, :5].all()
    assert rot_angle(pose[0, :, :3], opose[:, :3]) < 1e-6
    # exactly 4 points: the P3P gate passes, EPnP over all four (status / inliers as the oracle)
    st4, opose4, _, onin4, _ = O.pnp_ransac(s4[0], s4[1], s4[2], scale=1000.0)
    assert status[1] == st4 == 0 and nin[1] == onin4 == 4 and mask[1, :4].all()
    assert status[2] == P.STATUS_TOO_FEW and nin[2] == 0
    np.testing.assert_allclose(pose[2], np.eye(4)[:3])
    st6, opose6, omask6, onin6, _ = O.pnp_ransac(s6[0], s6[1], s6[2], scale=1000.0)
    assert status[3] == st6 and nin[3] == onin6


def test_drop_in_ransac_PnP(device):
    p2, p3, K, gt, inl = scene(3, 300, 0.25)
    pts3d_m = p3.astype(np.float64) / 1000.0
    pose, pose_homo, inliers = P.ransac_PnP(K, p2.astype(np.float64), pts3d_m, scale=1000)
    assert pose.shape == (3, 4) and pose_homo.shape == (4, 4)
    assert inliers.dtype == np.int32 and inliers.shape[1] == 1
    assert rot_angle(pose[:, :3], gt[:, :3]) < np.deg2rad(0.5)
    few = P.ransac_PnP(K, p2[:3], pts3d_m[:3], scale=1000)
    np.testing.assert_allclose(few[0], np.eye(4)[:3])
    assert few[2] == []


def test_four_point_p3p_gate_matches_oracle(device):
    """solvePnPRansac's 4-point branch on many scenes: exact, noisy, degenerate-looking ones (all
    image points on one pixel, solved by a far-away triangle; random sets, a few with no
    positive P3P root -> no model); status, inlier mask and count as the oracle's.  The pose
    of a 4-point solve is EPnP on a rank-deficient system (M is 8 x 12: a 4-dimensional null
    space), which amplifies rounding into degrees -- the oracle itself lands up to ~80 deg
    from the truth on exact data, and OpenCV's answer depends on its SVD -- so the pose is
    checked for form only: a finite rotation and translation."""
    scenes = [scene(200 + i, 4, 0.0 if i % 2 else 0.5) for i in range(12)]
    p2, p3, K, gt, inl = scene(7, 4, 0.0)
    scenes.append((np.repeat(p2[:1], 4, axis=0), p3, K, gt, inl))   # one pixel: a far solution
    rs = np.random.RandomState(5)
    for i in range(64):   # random 4-point sets: a few have no positive P3P solution
        q3 = rs.uniform(-100, 100, (4, 3)).astype(np.float32)
        q3[:, 2] += 400
        scenes.append((rs.uniform(0, 512, (4, 2)).astype(np.float32), q3, K, gt, inl))
    pose, mask, nin, status = run_gpu(scenes, device, max_points=4)
    n_fail = 0
    for b, (q2, q3, Kb, _, _) in enumerate(scenes):
        st, opose, omask, onin, _ = O.pnp_ransac(q2, q3, Kb, scale=1000.0)
        assert status[b] == st and nin[b] == onin, b
        np.testing.assert_array_equal(mask[b, :4], omask)
        assert np.isfinite(pose[b]).all()
        R = pose[b, :, :3]
        assert np.abs(R @ R.T - np.eye(3)).max() < 1e-9 and np.linalg.det(R) > 0
        if st != 0:
            np.testing.assert_array_equal(pose[b], np.eye(4)[:3])
        n_fail += st != 0
    assert 0 < n_fail < len(scenes)
