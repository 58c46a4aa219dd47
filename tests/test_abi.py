"""CPU tests of the C-ABI boundary: the library loads, exports every symbol the header
declares, and its host-side weight packer lays the reference weights out as documented."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO


def header_symbols():
    src = open(os.path.join(REPO, "include", "onepose_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(onepose_\w+)\s*\(", src)))


def test_header_declares_the_boundary():
    syms = header_symbols()
    for s in ["onepose_match", "onepose_matcher_pack", "onepose_pnp_ransac",
              "onepose_sample_descriptors", "onepose_select_correspondences",
              "onepose_pose_errors", "onepose_last_error"]:
        assert s in syms


def test_library_exports_every_header_symbol():
    from onepose_amd import _lib
    lib = _lib.load()
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert set(header_symbols()) == set(_lib.PROTOTYPES), "ctypes prototypes out of sync"
    assert lib.onepose_abi_version() == _lib.ABI_VERSION == 6


def test_object_cache_size_follows_its_flags():
    """The GAT prefix tables are reserved only when asked for and only for num_leaf <= 8,
    2 num_leaf rows of 1 KB per point and GAT layer plus 16 sorted logits (header)."""
    from onepose_amd import _lib
    lib = _lib.load()
    T = _lib.OBJ_GAT_TABLES
    for n3 in (1, 77, 4096):
        base = lib.onepose_object_cache_bytes(n3, 8, 0)
        for L in (1, 3, 8):
            assert lib.onepose_object_cache_bytes(n3, L, 0) == base
            assert lib.onepose_object_cache_bytes(n3, L, T) - base == 3 * n3 * (2 * L * 1024 + 64)
        assert lib.onepose_object_cache_bytes(n3, 12, T) == lib.onepose_object_cache_bytes(n3, 12, 0)
    # (+ 3 bf16 activation planes of the cached phi(q), 1.5 KB per point, in every precision)
    assert lib.onepose_object_cache_bytes(4096, 8, T) < 227.3e6
    assert lib.onepose_object_cache_bytes(4096, 8, 0) < 24.7e6
    assert lib.onepose_object_cache_bytes(0, 8, 0) == 0
    assert lib.onepose_object_cache_bytes(16, 17, 0) == 0
    assert lib.onepose_object_cache_bytes(16, 8, 2) == 0 and lib.onepose_object_cache_bytes(16, 8, -1) == 0


def test_tensor_list_matches_reference_state_dict():
    from onepose_amd import _lib, synthetic
    lib = _lib.load()
    sd = synthetic.make_state_dict(0)
    names = [lib.onepose_matcher_tensor_name(i).decode() for i in range(lib.onepose_matcher_num_tensors())]
    assert len(names) == 106
    for i, n in enumerate(names):
        assert n in sd, n
        assert sd[n].size == lib.onepose_matcher_tensor_numel(i)
    unused = set(sd) - set(names)
    assert all(k.startswith(("kenc_", "bin_score")) for k in unused)
    # the used parameter count quoted in SURVEY.md §8b
    assert sum(sd[n].size for n in names) == 5_587_200


def _pack(sd):
    from onepose_amd import _lib
    lib = _lib.load()
    names = [lib.onepose_matcher_tensor_name(i).decode() for i in range(lib.onepose_matcher_num_tensors())]
    host = [np.ascontiguousarray(sd[n], np.float32) for n in names]
    arr = (ctypes.c_void_p * len(host))(*[h.ctypes.data for h in host])
    buf = np.empty(lib.onepose_matcher_packed_bytes() // 4, np.float32)
    assert lib.onepose_matcher_pack(arr, len(host), buf.ctypes.data) == 0
    return buf


AP_FLOATS = 768 * 256 + 768 + 512 * 256 + 512 * 256 + 512 + 256 * 512 + 256 + 512 * 256


def test_pack_layout():
    """Packed panel of the first attention layer (gnn.layers.1), GAT fold, final proj."""
    from onepose_amd import synthetic
    sd = synthetic.make_state_dict(3)
    buf = _pack(sd)
    p = buf[:AP_FLOATS].astype(np.float64)
    off = 0

    def take(n):
        nonlocal off
        out = p[off:off + n]
        off += n
        return out
    wqkv = take(768 * 256).reshape(768, 256)
    bqkv = take(768)
    w1a = take(512 * 256).reshape(512, 256)
    cw = take(512 * 256).reshape(512, 256)
    b1 = take(512)
    w2 = take(256 * 512).reshape(256, 512)
    take(256)
    ct = take(512 * 256).reshape(256, 512)   # [h*64+q][o]
    q_w = sd["gnn.layers.1.attn.proj.0.weight"][:, :, 0]
    k_w = sd["gnn.layers.1.attn.proj.1.weight"][:, :, 0]
    v_w = sd["gnn.layers.1.attn.proj.2.weight"][:, :, 0]
    for h in range(4):
        for d in (0, 17, 63):
            np.testing.assert_array_equal(wqkv[h * 64 + d], q_w[d * 4 + h])
            np.testing.assert_array_equal(wqkv[256 + 128 * h + d], k_w[d * 4 + h])
            np.testing.assert_array_equal(wqkv[256 + 128 * h + 64 + d], v_w[d * 4 + h])
            assert bqkv[256 + 128 * h + 64 + d] == sd["gnn.layers.1.attn.proj.2.bias"][d * 4 + h]
            assert bqkv[h * 64 + d] == sd["gnn.layers.1.attn.proj.0.bias"][d * 4 + h]
    m0 = sd["gnn.layers.1.mlp.0.weight"][:, :, 0].astype(np.float64)
    merge = sd["gnn.layers.1.attn.merge.weight"][:, :, 0].astype(np.float64)
    np.testing.assert_array_equal(w1a, m0[:, :256])
    fold = m0[:, 256:] @ merge                       # columns in reference order q*4+h
    perm = np.array([(c % 64) * 4 + c // 64 for c in range(256)])
    np.testing.assert_allclose(cw, fold[:, perm], rtol=1e-5, atol=1e-6)
    b1f = sd["gnn.layers.1.mlp.0.bias"] + m0[:, 256:] @ sd["gnn.layers.1.attn.merge.bias"]
    np.testing.assert_allclose(b1, b1f, rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(w2, sd["gnn.layers.1.mlp.3.weight"][:, :, 0])
    np.testing.assert_array_equal(ct, cw.T)
    # bf16 planes of layer 1's Wqkv / W1a / W2 after the fp32 panel: hi = bf16 round-to-nearest-
    # even, hi + mid + lo == the fp32 weight exactly (the split gemm.hip applies to A on the fly)
    n_fp32 = 8 * AP_FLOATS + 4 * 512 + 256 * 256 + 256
    planes = buf[n_fp32:].view(np.uint16)
    assert planes.size == 8 * 3 * (768 * 256 + 512 * 256 + 256 * 512)

    def f32(b):
        return (b.astype(np.uint32) << 16).view(np.float32)
    po = 0
    for mat in (wqkv, w1a, w2):
        n = mat.size
        h, m, l = (planes[po + i * n:po + (i + 1) * n] for i in range(3))
        po += 3 * n
        x = mat.astype(np.float32).reshape(-1)
        u = x.view(np.uint32).astype(np.uint64)
        rne = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
        np.testing.assert_array_equal(h, rne)
        np.testing.assert_array_equal((f32(h) + f32(m)) + f32(l), x)
        assert np.all(np.abs(f32(l)) <= np.abs(x) * 2.0 ** -15 + 1e-38)
    # GAT fold: wa = W @ a (layer 0)
    gat0 = buf[8 * AP_FLOATS:8 * AP_FLOATS + 512]
    W, a = sd["gnn.layers.0.W"].astype(np.float64), sd["gnn.layers.0.a"][:, 0].astype(np.float64)
    np.testing.assert_allclose(gat0[:256], W @ a[:256], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(gat0[256:], W @ a[256:], rtol=1e-6, atol=1e-7)
    fin = buf[8 * AP_FLOATS + 4 * 512:]
    np.testing.assert_array_equal(fin[:65536], sd["final_proj.weight"].reshape(-1))


def test_pack_rejects_wrong_count():
    from onepose_amd import _lib
    lib = _lib.load()
    arr = (ctypes.c_void_p * 3)()
    assert lib.onepose_matcher_pack(arr, 3, None) != 0
    assert b"null" in lib.onepose_last_error() or b"expected" in lib.onepose_last_error()


def test_workspace_sizes():
    from onepose_amd import _lib
    lib = _lib.load()
    a = lib.onepose_match_workspace_bytes(1, 1024, 4096, 8, 1)
    b = lib.onepose_match_workspace_bytes(1, 1024, 4096, 8, 0)
    assert a > 0 and b - a >= 1024 * 4096 * 4
    assert lib.onepose_match_workspace_bytes(0, 1, 1, 8, 1) == 0
    # ABI 4: per precision -- fp32 carves no bf16 activation planes (x2 / x3 ping-pong and
    # phi(q), 3 planes of 512 B per token each: 6 KB per 2D + 3D token pair ... per token)
    from onepose_amd.matcher import PRECISIONS
    for B, n1, n3 in ((1, 1024, 4096), (3, 200, 330)):
        full = lib.onepose_match_workspace_bytes(B, n1, n3, 8, 1)
        f32 = lib.onepose_match_workspace_bytes_ex(B, n1, n3, 8, 1, PRECISIONS["fp32"])
        assert lib.onepose_match_workspace_bytes_ex(B, n1, n3, 8, 1, PRECISIONS["bf16"]) == full
        assert lib.onepose_match_workspace_bytes_ex(B, n1, n3, 8, 1, PRECISIONS["fp32_split"]) == full
        planes = 3 * 3 * 256 * 2 * B * (n1 + n3)   # (x ping, x pong, phi(q)) x 3 planes x bf16
        assert 0 <= full - f32 - planes < 3 * 256 * 8
    assert lib.onepose_match_workspace_bytes_ex(1, 8, 8, 8, 1, 7) == 0


def test_object_cache_size_per_precision():
    from onepose_amd import _lib
    from onepose_amd.matcher import PRECISIONS
    lib = _lib.load()
    for flags in (0, _lib.OBJ_GAT_TABLES):
        for n3 in (77, 4096):
            full = lib.onepose_object_cache_bytes(n3, 8, flags)
            assert lib.onepose_object_cache_bytes_ex(n3, 8, flags, PRECISIONS["bf16"]) == full
            assert lib.onepose_object_cache_bytes_ex(n3, 8, flags, PRECISIONS["fp32_split"]) == full
            assert full - lib.onepose_object_cache_bytes_ex(n3, 8, flags, PRECISIONS["fp32"]) == 1536 * n3
    assert lib.onepose_object_cache_bytes_ex(16, 8, 0, 9) == 0
    assert lib.onepose_pnp_workspace_bytes(2, 1024, 10000) >= 2 * 1024 * 4


def test_module_state_dict_keys_match_reference():
    """The drop-in module accepts the reference's full state dict (strict)."""
    from onepose_amd import matcher, synthetic
    sd = synthetic.make_state_dict(0)
    m = matcher.from_state_dict(sd)
    assert set(m.state_dict().keys()) == set(sd.keys())
    assert sum(p.numel() for p in m.parameters()) == 5_674_401


def test_empty_input_path_matches_reference():
    """GATs_SuperGlue.py:223-231 -- a bare dict with int32 indices (golden from the reference)."""
    import torch
    from conftest import golden
    from onepose_amd import matcher, synthetic
    g = golden("matcher_empty")
    m = matcher.from_state_dict(synthetic.make_state_dict(0))
    out = m({"keypoints2d": torch.zeros(1, 0, 2), "keypoints3d": torch.zeros(1, 5, 3),
             "descriptors2d_query": torch.zeros(1, 256, 0), "descriptors3d_db": torch.zeros(1, 256, 5),
             "descriptors2d_db": torch.zeros(1, 256, 40)})
    assert isinstance(out, dict) and out["skip_train"] is True
    for k in ("matches0", "matches1", "matching_scores0", "matching_scores1"):
        assert out[k].numpy().dtype == g[k].dtype
        np.testing.assert_array_equal(out[k].numpy(), g[k])


def test_cpu_forward_fails_loudly():
    import torch
    from onepose_amd import matcher, synthetic
    m = matcher.from_state_dict(synthetic.make_state_dict(0))
    data, _, _ = synthetic.make_matcher_inputs(16, 8, 2, seed=0)
    with pytest.raises(RuntimeError, match="GPU"):
        m({k: torch.from_numpy(v) for k, v in data.items()})


def test_unsupported_match_type():
    import torch
    from onepose_amd import matcher, synthetic
    hp = dict(synthetic.DEFAULT_HPARAMS, match_type="sinkhorn")
    m = matcher.from_state_dict(synthetic.make_state_dict(0), hp)
    data, _, _ = synthetic.make_matcher_inputs(16, 8, 2, seed=0)
    with pytest.raises(NotImplementedError):
        m({k: torch.from_numpy(v) for k, v in data.items()})


def test_match_cached_stages_rejects_bad_ranges():
    """onepose_match_cached_stages (ABI 6) runs a range of the forward's stages; an empty or
    out-of-order range is refused before any argument is touched (no device needed)."""
    from onepose_amd import _lib
    lib = _lib.load()
    assert (_lib.STAGE_INPUTS, _lib.STAGE_LAYER0, _lib.STAGE_FINAL, _lib.STAGE_SCORE,
            _lib.STAGE_WINNERS) == (0, 1, 13, 14, 15)
    for first, last in ((-1, 15), (0, 16), (5, 4), (15, 14), (16, 16)):
        rc = lib.onepose_match_cached_stages(None, None, 0, 0, None, None, 0, 1, 8, 8, 8, 1.0,
                                             0.2, 0, 0, None, None, None, None, None, None, 0,
                                             first, last, None)
        assert rc != 0
        assert b"stages" in lib.onepose_last_error()
