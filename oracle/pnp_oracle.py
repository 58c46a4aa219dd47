"""ORACLE -- test infrastructure only.  ctypes loader for oracle/liboracle.so (built from
oracle/epnp_ransac.c by ``onepose_amd.build.build_oracle``).  Only tests/, smoke() and
bench.py's cpu_baseline leg may use it."""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            import sys
            sys.path.insert(0, os.path.dirname(HERE))
            from onepose_amd.build import build_oracle
            build_oracle()
        lib = ctypes.CDLL(LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        fp = ctypes.POINTER(ctypes.c_float)
        lib.oracle_pnp_ransac.restype = ctypes.c_int
        lib.oracle_pnp_ransac.argtypes = [fp, fp, ctypes.c_int, dp, ctypes.c_double, ctypes.c_float,
                                          ctypes.c_int, ctypes.c_double, dp,
                                          ctypes.POINTER(ctypes.c_ubyte),
                                          ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        lib.oracle_epnp.restype = None
        lib.oracle_epnp.argtypes = [dp, dp, ctypes.c_int, dp, dp, dp]
        lib.oracle_rng_draws.restype = None
        lib.oracle_rng_draws.argtypes = [ctypes.POINTER(ctypes.c_uint), ctypes.c_int]
        lib.oracle_p3p_solutions.restype = ctypes.c_int
        lib.oracle_p3p_solutions.argtypes = [fp, fp, dp]
        lib.oracle_rodrigues_m2v.argtypes = [dp, dp]
        lib.oracle_rodrigues_v2m.argtypes = [dp, dp]
        _lib = lib
    return _lib


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def p3p_solutions(pts2d_f32, pts3d_f32, K):
    """Number of P3P solutions from the first three correspondences (the 4-point gate)."""
    p2 = np.ascontiguousarray(pts2d_f32, np.float32)
    p3 = np.ascontiguousarray(pts3d_f32, np.float32)
    Kd = np.ascontiguousarray(K, np.float64)
    return int(load().oracle_p3p_solutions(_p(p2, ctypes.c_float), _p(p3, ctypes.c_float),
                                           _p(Kd, ctypes.c_double)))


def pnp_ransac(pts2d_f32, pts3d_f32, K, scale=1.0, reproj=5.0, max_iters=10000, confidence=0.99):
    """Returns (status, pose34 [3,4], mask [n] bool, n_inliers, iterations_run)."""
    lib = load()
    p2 = np.ascontiguousarray(pts2d_f32, dtype=np.float32).reshape(-1, 2)
    p3 = np.ascontiguousarray(pts3d_f32, dtype=np.float32).reshape(-1, 3)
    n = p2.shape[0]
    K = np.ascontiguousarray(K, dtype=np.float64).reshape(9)
    pose = np.zeros(12, np.float64)
    mask = np.zeros(max(n, 1), np.uint8)
    nin = ctypes.c_int(0)
    iters = ctypes.c_int(0)
    st = lib.oracle_pnp_ransac(_p(p2, ctypes.c_float), _p(p3, ctypes.c_float), n,
                               _p(K, ctypes.c_double), scale, reproj, max_iters, confidence,
                               _p(pose, ctypes.c_double), _p(mask, ctypes.c_ubyte),
                               ctypes.byref(nin), ctypes.byref(iters))
    return st, pose.reshape(3, 4), mask[:n].astype(bool), nin.value, iters.value


def epnp(pws, us, K):
    lib = load()
    pws = np.ascontiguousarray(pws, np.float64).reshape(-1, 3)
    us = np.ascontiguousarray(us, np.float64).reshape(-1, 2)
    K = np.ascontiguousarray(K, np.float64).reshape(9)
    R = np.zeros(9)
    t = np.zeros(3)
    lib.oracle_epnp(_p(pws, ctypes.c_double), _p(us, ctypes.c_double), pws.shape[0],
                    _p(K, ctypes.c_double), _p(R, ctypes.c_double), _p(t, ctypes.c_double))
    return R.reshape(3, 3), t


def rng_draws(count):
    lib = load()
    out = np.zeros(count, np.uint32)
    lib.oracle_rng_draws(out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint)), count)
    return out


def select_correspondences(matches0, kpts2d, kpts3d, scale=1.0):
    """inference.py:147-152 + eval_utils.py:22-26 + solvePnPRansac's float32 conversion."""
    valid = matches0 > -1
    p2 = np.asarray(kpts2d, np.float32)[valid]
    p3 = (np.asarray(kpts3d, np.float32)[matches0[valid]].astype(np.float64) * scale).astype(np.float32)
    return p2, p3


def pose_error(pose_pred, pose_gt):
    """eval_utils.query_pose_error restated."""
    pose_pred = np.asarray(pose_pred)[:3]
    pose_gt = np.asarray(pose_gt)[:3]
    t = np.linalg.norm(pose_pred[:, 3] - pose_gt[:, 3]) * 100
    tr = np.trace(pose_pred[:, :3] @ pose_gt[:, :3].T)
    tr = tr if tr <= 3 else 3
    return np.rad2deg(np.arccos((tr - 1.0) / 2.0)), t
