"""Known-answer tests of the C RANSAC-EPnP oracle (oracle/epnp_ransac.c), CPU only.

The reference solves pose with cv2.solvePnPRansac(SOLVEPNP_EPNP) (eval_utils.py:18-42,
opencv_python==4.4.0.46 per requirements.txt:5).  cv2 is not installed and cannot be, so
the oracle is parity-unpinned against OpenCV itself; these tests pin it on scenes with a
known answer: exact data must give the ground-truth pose and the true inlier
set, noisy data the noise-limited pose, too few points a failure status, and the random
stream is the published cv::RNG multiply-with-carry recurrence."""
import numpy as np
import pytest

from onepose_amd import synthetic as S
from oracle import pnp_oracle as O


def scene(seed, n, outlier_frac=0.3, px_noise=0.0):
    rs = np.random.RandomState(seed)
    K = S.crop_intrinsics()
    R = S.random_rotation(rs)
    t = np.array([rs.uniform(-0.03, 0.03), rs.uniform(-0.03, 0.03), rs.uniform(0.35, 0.55)])
    pose = np.concatenate([R, t[:, None]], 1)
    pts = rs.uniform(-0.1, 0.1, (n, 3)).astype(np.float32)
    uv = S.project(K, pose, pts.astype(np.float64)) + rs.normal(0, px_noise, (n, 2))
    out = rs.rand(n) < outlier_frac
    uv[out] = rs.uniform(0, 512, (out.sum(), 2))
    # a random outlier can land within the 5 px gate by chance; those are inliers by definition
    near = np.linalg.norm(uv - S.project(K, pose, pts.astype(np.float64)), axis=1) <= 5.0
    return uv.astype(np.float32), pts, K, pose, near


def rot_err(Ra, Rb):
    return np.arccos(np.clip((np.trace(Ra @ Rb.T) - 1) / 2, -1, 1))


def test_cv_rng_stream():
    """cv::RNG((uint64)-1): state = (u32)state * 4164903690 + (state >> 32), draw = (u32)state."""
    state = 0xFFFFFFFFFFFFFFFF
    want = []
    for _ in range(64):
        state = ((state & 0xFFFFFFFF) * 4164903690 + (state >> 32)) & 0xFFFFFFFFFFFFFFFF
        want.append(state & 0xFFFFFFFF)
    np.testing.assert_array_equal(O.rng_draws(64), np.array(want, np.uint32))


@pytest.mark.parametrize("n", [6, 12, 50])
def test_epnp_exact_correspondences(n):
    p2, p3, K, pose, _ = scene(11 + n, n, outlier_frac=0.0)
    R, t = O.epnp(p3.astype(np.float64), p2.astype(np.float64), K)
    assert rot_err(R, pose[:, :3]) < 1e-5
    assert np.linalg.norm(t - pose[:, 3]) < 1e-5


@pytest.mark.parametrize("seed,outliers", [(1, 0.0), (2, 0.3), (3, 0.6)])
def test_ransac_exact_scene_recovers_pose_and_inliers(seed, outliers):
    p2, p3, K, pose, near = scene(seed, 400, outlier_frac=outliers)
    st, est, mask, nin, _ = O.pnp_ransac(p2, p3 * 1000.0, K, scale=1000.0)
    assert st == 0
    np.testing.assert_array_equal(mask, near)
    assert nin == near.sum()
    assert rot_err(est[:, :3], pose[:, :3]) < 1e-4       # north-star bound, radians
    assert np.linalg.norm(est[:, 3] - pose[:, 3]) < 1e-3


def test_ransac_noisy_scene_is_noise_limited():
    p2, p3, K, pose, near = scene(7, 700, outlier_frac=0.3, px_noise=0.5)
    st, est, mask, nin, _ = O.pnp_ransac(p2, p3 * 1000.0, K, scale=1000.0)
    assert st == 0
    assert (mask & ~near).sum() <= 2                      # essentially no gross outliers kept
    assert (near & mask).sum() >= 0.97 * near.sum()
    assert np.degrees(rot_err(est[:, :3], pose[:, :3])) < 0.5
    assert np.linalg.norm(est[:, 3] - pose[:, 3]) < 5e-3


def test_ransac_too_few_points_fails():
    p2, p3, K, _, _ = scene(5, 3, outlier_frac=0.0)
    st, est, mask, nin, _ = O.pnp_ransac(p2, p3 * 1000.0, K, scale=1000.0)
    assert st != 0 and nin == 0


def test_four_points_take_the_p3p_gate():
    """Exactly 4 correspondences: cv::solvePnPRansac switches to model_points 4 with the P3P
    kernel, which (count == model_points) runs once; a model means all four are inliers and
    the final refit is EPnP over them.  The true lengths are among P3P's solutions; one image
    point for all four rays has no solution and fails."""
    for seed in range(4):
        p2, p3, K, pose, _ = scene(100 + seed, 4, outlier_frac=0.0)
        assert O.p3p_solutions(p2, p3 * 1000.0, K) >= 1
        st, est, mask, nin, _ = O.pnp_ransac(p2, p3 * 1000.0, K, scale=1000.0)
        assert st == 0 and nin == 4 and mask.all()
        R, t = np.zeros(9), np.zeros(3)
        O.load().oracle_epnp(O._p(np.ascontiguousarray(p3 * 1000.0, np.float64), O.ctypes.c_double),
                             O._p(np.ascontiguousarray(p2, np.float64), O.ctypes.c_double), 4,
                             O._p(np.ascontiguousarray(K, np.float64), O.ctypes.c_double),
                             O._p(R, O.ctypes.c_double), O._p(t, O.ctypes.c_double))
        assert rot_err(est[:, :3], R.reshape(3, 3)) < 1e-6   # the EPnP refit of all four
    p2, p3, K, _, _ = scene(7, 4, outlier_frac=0.0)
    p2[:] = p2[0]
    assert O.p3p_solutions(p2, p3 * 1000.0, K) == 0
    st, est, _, nin, _ = O.pnp_ransac(p2, p3 * 1000.0, K, scale=1000.0)
    assert st == 2 and nin == 0 and np.allclose(est, np.eye(4)[:3])


def test_p3p_quartic_recovers_true_lengths():
    """The gate's quartic has the true distance ratio x = |P0|/|P2| among its positive roots:
    a known-answer check of the elimination (restated from Gao et al., not from OpenCV)."""
    for seed in range(6):
        p2, p3, K, pose, _ = scene(300 + seed, 4, outlier_frac=0.0)
        Pc = (pose[:, :3] @ p3.astype(np.float64).T).T + pose[:, 3]
        d = np.linalg.norm(Pc, axis=1)
        bear = Pc / d[:, None]
        # the law-of-cosines system the gate solves, at the true lengths
        x, y = d[0] / d[2], d[1] / d[2]
        p, q, r = 2 * bear[1] @ bear[2], 2 * bear[0] @ bear[2], 2 * bear[0] @ bear[1]
        dd = lambda i, j: np.linalg.norm(p3[i].astype(np.float64) - p3[j])
        a, b = dd(1, 2) ** 2 / dd(0, 1) ** 2, dd(0, 2) ** 2 / dd(0, 1) ** 2
        assert abs((1 - a) * y * y + (a * x * r - p) * y + (1 - a * x * x)) < 1e-9
        assert abs(-b * y * y + b * x * r * y + ((1 - b) * x * x - q * x + 1)) < 1e-9
        assert O.p3p_solutions(p2, p3 * 1000.0, K) >= 1


def test_pose_error_semantics():
    """query_pose_error (eval_utils.py:45-63): cm and degrees, trace clamped at 3 only."""
    R = S.random_rotation(np.random.RandomState(0))
    gt = np.concatenate([R, np.array([[0.0], [0.0], [0.5]])], 1)
    pr = gt.copy()
    pr[2, 3] += 0.02
    r, t = O.pose_error(pr, gt)
    assert abs(t - 2.0) < 1e-9 and r < 1e-4


def test_mwc_jump_ahead_identity():
    """cv::RNG's multiply-with-carry step s' = (s mod 2^32) * A + (s >> 32) is, for states
    below m = A * 2^32 - 1, multiplication by A mod m -- the identity the GPU RANSAC uses to
    generate a round's draws in parallel (lane l starts at A^(6 l) z mod m).  RNG((uint64)-1)
    starts above m: the first two draws are stepped one by one (pnp.hip kRngPrefix)."""
    A = 4164903690
    m = A * 2**32 - 1

    def step(s):
        return (s & 0xFFFFFFFF) * A + (s >> 32)

    z, seq = 2**64 - 1, []
    for _ in range(800):
        z = step(z)
        seq.append(z)
    first = next(i for i, v in enumerate(seq) if v < m)
    assert first == 1 and all(v < m for v in seq[first:])
    for k in (1, 5, 6, 64, 384, 700):
        assert seq[first + k] == pow(A, k, m) * seq[first] % m
