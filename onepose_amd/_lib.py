"""ctypes binding of libonepose_hip.so (the C-ABI in include/onepose_hip.h).

This is the binding a maintainer of the reference would drop in: plain
pointers from ``torch.Tensor.data_ptr()``, the current HIP stream, and an int status mapped
to exceptions.  The library is loaded from the package directory (built in-tree by
``onepose_amd.build``); there is no fallback -- if it is missing, every call raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# ONEPOSE_LIB: an alternative in-tree build of the same library (A/B measurement, tools/ab.sh)
LIB_PATH = os.environ.get("ONEPOSE_LIB") or os.path.join(_HERE, "libonepose_hip.so")

c_int, c_int64, c_size_t, c_float, c_double = (ctypes.c_int, ctypes.c_int64, ctypes.c_size_t,
                                               ctypes.c_float, ctypes.c_double)
c_void_p, c_char_p = ctypes.c_void_p, ctypes.c_char_p

# onepose_allgather_fn: int (*)(size_t bytes_per_rank, void* stream, void* user)
ALLGATHER_FN = ctypes.CFUNCTYPE(c_int, c_size_t, c_void_p, c_void_p)
ABI_VERSION = 6
DEVERR_STALE_CACHE = 1   # ONEPOSE_DEVERR_STALE_CACHE
STAGE_INPUTS, STAGE_LAYER0, STAGE_FINAL, STAGE_SCORE, STAGE_WINNERS = 0, 1, 13, 14, 15  # ABI 6
OBJ_GAT_TABLES = 1   # ONEPOSE_OBJ_GAT_TABLES
DT_F32, DT_F16 = 0, 1   # ONEPOSE_DT_*

# name -> (restype, argtypes); mirrors include/onepose_hip.h
PROTOTYPES = {
    "onepose_last_error": (c_char_p, []),
    "onepose_abi_version": (c_int, []),
    "onepose_device_errors": (c_int, [c_int, ctypes.POINTER(ctypes.c_uint)]),
    "onepose_matcher_num_tensors": (c_int, []),
    "onepose_matcher_tensor_name": (c_char_p, [c_int]),
    "onepose_matcher_tensor_numel": (c_int64, [c_int]),
    "onepose_matcher_packed_bytes": (c_size_t, []),
    "onepose_matcher_pack": (c_int, [ctypes.POINTER(c_void_p), c_int, c_void_p]),
    "onepose_match_workspace_bytes": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "onepose_match_workspace_bytes_ex": (c_size_t, [c_int, c_int, c_int, c_int, c_int, c_int]),
    "onepose_prepare_leaves_dt": (c_int, [c_void_p, c_int, c_int64, c_int, c_int, c_int, c_void_p,
                                          c_void_p]),
    "onepose_match_dt": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64,
                                 c_int, c_int, c_int, c_int, c_int, c_float, c_float, c_int,
                                 c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_size_t, c_void_p]),
    "onepose_object_prepare_dt": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int,
                                          c_int, c_void_p, c_void_p, c_size_t, c_void_p]),
    "onepose_match_cached_dt": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_void_p, c_void_p,
                                        c_int64, c_int, c_int, c_int, c_int, c_float, c_float,
                                        c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p, c_void_p, c_size_t, c_void_p]),
    "onepose_match_cached_stages": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_void_p,
                                            c_void_p, c_int64, c_int, c_int, c_int, c_int,
                                            c_float, c_float, c_int, c_int, c_void_p, c_void_p,
                                            c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                            c_int, c_int, c_void_p]),
    "onepose_match": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64,
                              c_int, c_int, c_int, c_int, c_float, c_float,
                              c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                              c_void_p, c_size_t, c_void_p]),
    "onepose_match_prepared": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p,
                                       c_int64, c_int, c_int, c_int, c_int, c_float, c_float,
                                       c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_size_t, c_void_p]),
    "onepose_match_ex": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p,
                                 c_int64, c_int, c_int, c_int, c_int, c_float, c_float, c_int,
                                 c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_size_t, c_void_p]),
    "onepose_match_prepared_ex": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_int64,
                                          c_void_p, c_int64, c_int, c_int, c_int, c_int, c_float,
                                          c_float, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                          c_void_p, c_void_p, c_size_t, c_void_p]),
    "onepose_object_cache_bytes": (c_size_t, [c_int, c_int, c_int]),
    "onepose_object_cache_bytes_ex": (c_size_t, [c_int, c_int, c_int, c_int]),
    "onepose_object_prepare_workspace_bytes": (c_size_t, [c_int, c_int]),
    "onepose_object_prepare": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                       c_int, c_void_p, c_void_p, c_size_t, c_void_p]),
    "onepose_object_release": (None, [c_void_p]),
    "onepose_match_cached": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int64,
                                     c_int, c_int, c_int, c_int, c_float, c_float, c_int, c_int,
                                     c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                     c_void_p, c_size_t, c_void_p]),
    "onepose_shard_range": (None, [c_int, c_int, c_int, ctypes.POINTER(c_int),
                                   ctypes.POINTER(c_int)]),
    "onepose_match_sharded_xchg_bytes": (c_size_t, [c_int, c_int, c_int, c_int]),
    "onepose_match_sharded_workspace_bytes": (c_size_t, [c_int, c_int, c_int, c_int, c_int,
                                                         c_int, c_int]),
    "onepose_match_sharded": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p,
                                      c_int64, c_int, c_int, c_int, c_int, c_int, c_int,
                                      c_float, c_float, c_int, c_void_p, c_void_p, c_size_t,
                                      ALLGATHER_FN, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "onepose_leaves_prepared_bytes": (c_size_t, [c_int, c_int, c_int]),
    "onepose_prepare_leaves": (c_int, [c_void_p, c_int64, c_int, c_int, c_int, c_void_p,
                                       c_void_p]),
    "onepose_sample_descriptors": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                           c_int, c_int, c_void_p, c_void_p]),
    "onepose_select_correspondences": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_int64,
                                               c_int, c_int, c_int, c_double, c_void_p, c_void_p,
                                               c_void_p, c_void_p]),
    "onepose_pnp_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
    "onepose_pnp_ransac": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int64, c_int,
                                   c_double, c_float, c_int, c_double, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "onepose_pose_errors": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_void_p, c_void_p,
                                    c_void_p, c_void_p]),
    "onepose_pose_stage": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_int, c_int,
                                   c_int, c_double, c_void_p, c_int64, c_float, c_int, c_double,
                                   c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_size_t, c_void_p]),
    "onepose_superpoint_num_tensors": (c_int, []),
    "onepose_superpoint_tensor_name": (c_char_p, [c_int]),
    "onepose_superpoint_packed_bytes": (c_size_t, []),
    "onepose_superpoint_pack": (c_int, [ctypes.POINTER(c_void_p), c_int, c_void_p]),
    "onepose_superpoint_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
    "onepose_superpoint": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float, c_int,
                                   c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_size_t, c_void_p]),
    "onepose_superpoint_detect_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
    "onepose_superpoint_detect": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float,
                                          c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                          c_void_p, c_void_p, c_size_t, c_void_p]),
    "onepose_profile_begin": (c_int, [ctypes.c_uint64, c_int]),
    "onepose_profile_begin_device": (c_int, [ctypes.c_uint64]),
    "onepose_profile_end_device": (c_int, [c_void_p, c_void_p, c_int]),
    "onepose_profile_end": (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    "onepose_profile_kind_name": (c_char_p, [c_int]),
}

_lib = None


class OnePoseError(RuntimeError):
    pass


def load():
    """Load the shared library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OnePoseError(
                f"{LIB_PATH} is missing: build it with `python -m onepose_amd.build` "
                "(onepose_amd has no CPU fallback)")
        lib = ctypes.CDLL(LIB_PATH)
        # A/B measurement only: an older build named by ONEPOSE_LIB may predate the newest
        # entry points (ABI >= 3); callers fall back where one is missing (size_query)
        ab = bool(os.environ.get("ONEPOSE_LIB"))
        for name, (res, args) in PROTOTYPES.items():
            if ab and not hasattr(lib, name):
                continue
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.onepose_abi_version() != ABI_VERSION and not (ab and lib.onepose_abi_version() >= 3):
            raise OnePoseError(f"{LIB_PATH}: ABI version {lib.onepose_abi_version()}, "
                               f"expected {ABI_VERSION}: rebuild with `python -m onepose_amd.build`")
        _lib = lib
    return _lib


def workspace_bytes(lib, B, n1, n3, L, with_conf, precision) -> int:
    """onepose_match_workspace_bytes_ex (this precision's need), or the every-precision query
    on an older A/B build without it."""
    if hasattr(lib, "onepose_match_workspace_bytes_ex"):
        return lib.onepose_match_workspace_bytes_ex(B, n1, n3, L, int(with_conf), int(precision))
    return lib.onepose_match_workspace_bytes(B, n1, n3, L, int(with_conf))


def object_cache_bytes(lib, n3, L, flags, precision) -> int:
    if hasattr(lib, "onepose_object_cache_bytes_ex"):
        return lib.onepose_object_cache_bytes_ex(n3, L, flags, int(precision))
    return lib.onepose_object_cache_bytes(n3, L, flags)


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = load().onepose_last_error().decode(errors="replace")
        raise OnePoseError(f"{what or 'onepose_hip'} failed (status {rc}): {msg}")


def stream_ptr(device=None) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def device_errors(clear: bool = False) -> int:
    """The library's sticky device-side error bits (DEVERR_*; onepose_device_errors).
    Synchronises with the device."""
    lib = load()
    v = ctypes.c_uint(0)
    check(lib.onepose_device_errors(1 if clear else 0, ctypes.byref(v)), "device_errors")
    return int(v.value)
