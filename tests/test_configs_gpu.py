"""BASELINE configs 3 and 4 at their own batch (GATs_SuperGlue.py:203-278), through the bench's
path: the object prepared once (onepose_object_prepare with the GAT prefix tables), then
onepose_match_cached over the whole batch.

  config 3: 1024 kpts x 16384 3D pts, B = 32.  Frame 0 of the batch is the reference-generated
            fixture matcher_c3_idx (make_golden.py): indices exact, scores within 2e-5
            (tests/parity.py).  Frames 1, 17 and 31 equal their own B = 1 runs (same contract:
            the batch takes other tiles -- 128-row QKV, 64x64 MLP conv 2, kv_reduce + m_fold --
            so only the summation order differs).
  config 4: 1024 x 2500 (ragged: 2500 = 39 x 64 + 4), B = 32, the per-GPU shard of the 8-GPU
            sweep.  Frames 0 and 31 against the numpy oracle (oracle/matcher_np.py, pinned to the
            reference's fixtures by test_oracle_golden.py): conf within 2e-5, indices exact.
The batch's per-object tensors are shared (batch stride 0), as the pipeline runs them."""
import numpy as np
import pytest
import torch

from conftest import golden
from onepose_amd import _lib, matcher, synthetic
from parity import ATOL, assert_pred_equal

pytestmark = pytest.mark.gpu


def batch_inputs(n1, n3, L, seed, B):
    """One object (batch 1 arrays) and B frames of it: frame b is make_matcher_inputs'
    frame b for the same seed, so frame 0 is the fixture's frame."""
    data, obj, _ = synthetic.make_matcher_inputs(n1, n3, L, seed=seed, batch=1)
    frames = [synthetic.make_frame(obj, n1, seed * 131 + b) for b in range(B)]
    d2 = np.stack([f.descriptors2d for f in frames])
    return data, d2


class CachedMatcher:
    """onepose_object_prepare once + onepose_match_cached per call (the FramePipeline path)."""

    def __init__(self, sd, data, device, flags=_lib.OBJ_GAT_TABLES, precision=0, fp16=False):
        """fp16: the object's descriptors and leaves and every query's descriptors go to the
        library as fp16 (the _dt entry points)."""
        self.lib = lib = _lib.load()
        self.device, self.flags, self.precision = device, flags, precision
        self.dt = _lib.DT_F16 if fp16 else _lib.DT_F32
        ddt = np.float16 if fp16 else np.float32
        m = matcher.from_state_dict(sd)
        self.sf = float(m.hparams["scale_factor"])
        self.thr = float(m.hparams["match_threshold"])
        self.w = m.packed_weights(device)
        f32 = dict(dtype=torch.float32, device=device)
        self.n3 = n3 = data["descriptors3d_db"].shape[2]
        self.L = L = data["descriptors2d_db"].shape[2] // n3
        d3 = torch.from_numpy(data["descriptors3d_db"][0].astype(ddt)).to(device).contiguous()
        lv = torch.from_numpy(data["descriptors2d_db"][0].astype(ddt)).to(device).contiguous()
        s = _lib.stream_ptr(device)
        self.pm = torch.empty(lib.onepose_leaves_prepared_bytes(1, n3, L) // 4, **f32)
        _lib.check(lib.onepose_prepare_leaves_dt(lv.data_ptr(), self.dt, 0, 1, n3, L,
                                                 self.pm.data_ptr(), s), "leaves")
        self.cache = torch.empty(
            _lib.object_cache_bytes(lib, n3, L, flags, precision) // 4, **f32)
        wsb = lib.onepose_object_prepare_workspace_bytes(n3, L)
        ws = torch.empty(wsb, dtype=torch.uint8, device=device)
        _lib.check(lib.onepose_object_prepare_dt(self.w.data_ptr(), d3.data_ptr(), self.dt,
                                                 self.pm.data_ptr(), n3, L, precision, flags,
                                                 self.cache.data_ptr(), ws.data_ptr(), wsb, s),
                   "prepare")
        torch.cuda.synchronize()

    def __del__(self):   # drop the library's record of the cache with its memory
        cache = self.__dict__.get("cache")
        if cache is not None:
            self.lib.onepose_object_release(cache.data_ptr())

    def __call__(self, d2, with_conf=False):
        """d2 [B, 256, n1] numpy -> per-frame pred dicts (and conf [B, n1, n3] if asked)."""
        lib, dev = self.lib, self.device
        B, _, n1 = d2.shape
        n3 = self.n3
        f32 = dict(dtype=torch.float32, device=dev)
        t = torch.from_numpy(np.ascontiguousarray(
            d2.astype(np.float16 if self.dt == _lib.DT_F16 else np.float32))).to(dev)
        o = dict(m0=torch.empty(B, n1, dtype=torch.int64, device=dev),
                 m1=torch.empty(B, n3, dtype=torch.int64, device=dev),
                 s0=torch.empty(B, n1, **f32), s1=torch.empty(B, n3, **f32))
        conf = torch.empty(B, n1, n3, **f32) if with_conf else None
        wsb = _lib.workspace_bytes(lib, B, n1, n3, self.L, with_conf, self.precision)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        _lib.check(lib.onepose_match_cached_dt(
            self.w.data_ptr(), t.data_ptr(), self.dt, 256 * n1, self.cache.data_ptr(),
            self.pm.data_ptr(),
            0, B, n1, n3, self.L, self.sf, self.thr, self.precision, self.flags,
            o["m0"].data_ptr(), o["m1"].data_ptr(), o["s0"].data_ptr(), o["s1"].data_ptr(),
            _lib.ptr(conf), ws.data_ptr(), wsb, _lib.stream_ptr(dev)), "match_cached")
        torch.cuda.synchronize()
        h = {k: v.cpu().numpy() for k, v in o.items()}
        preds = [{"matches0": h["m0"][b], "matches1": h["m1"][b], "matching_scores0": h["s0"][b],
                  "matching_scores1": h["s1"][b]} for b in range(B)]
        return preds, (conf.cpu().numpy() if with_conf else None)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("precision", [0, 2], ids=["fp32", "fp32_split"])
def test_config3_batch32_1024x16384(device, precision):
    g = golden("matcher_c3_idx")
    n1, n3, L, seed = [int(g[k]) for k in ("n1", "n3", "num_leaf", "seed")]
    assert (n1, n3, L) == (1024, 16384, 8)
    sd = synthetic.make_state_dict(seed, well_conditioned=bool(int(g["well_conditioned"])))
    data, d2 = batch_inputs(n1, n3, L, seed, 32)
    cm = CachedMatcher(sd, data, device, precision=precision)
    preds, _ = cm(d2)
    assert_pred_equal(preds[0], g, "config 3, frame 0 of 32 vs the reference")
    for b in (1, 17, 31):
        one, _ = cm(d2[b:b + 1])
        assert_pred_equal(preds[b], one[0], f"config 3, frame {b} of 32 vs alone")
        assert (preds[b]["matches0"] > -1).sum() > 200
    # mutual consistency over the whole batch
    for p in preds:
        m0, m1 = p["matches0"], p["matches1"]
        ok = m0 > -1
        assert np.array_equal(m1[m0[ok]], np.nonzero(ok)[0])
        assert (m1 > -1).sum() == ok.sum()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("precision", [0, 2], ids=["fp32", "fp32_split"])
def test_config4_batch32_1024x2500_ragged(device, precision):
    """Config 4's per-GPU shard (B = 32, ragged n3 = 2500) through the cached path, frames 0
    and 31 against the numpy oracle under the index contract -- in fp32 and in the split mode
    (its batched launches: 64 x 128 QKV tiles, the separate m_fold with bf16 planes)."""
    from oracle import matcher_np as M
    n1, n3, L, seed = 1024, 2500, 8, 12
    sd = synthetic.make_state_dict(seed)
    data, d2 = batch_inputs(n1, n3, L, seed, 32)
    cm = CachedMatcher(sd, data, device, precision=precision)
    preds, conf = cm(d2, with_conf=True)
    for b in (0, 31):
        one = dict(data)
        one["descriptors2d_query"] = d2[b:b + 1]
        opred, oconf = M.forward(sd, one)
        np.testing.assert_allclose(conf[b], oconf[0], rtol=0, atol=ATOL)
        assert_pred_equal(preds[b], opred, f"config 4, frame {b} of 32 vs oracle")
        assert (preds[b]["matches0"] > -1).sum() > 200


@pytest.mark.timeout(300)
def test_config5_2048x8192_vs_oracle(device):
    """BASELINE config 5 shape (2048 kpts x 8192 3D pts, L = 8) through the bench's cached path,
    anchored to the numpy oracle (oracle/matcher_np.py, pinned to the reference fixtures):
      fp32: conf within 2e-5 and indices exact (tests/parity.py);
      bf16 attention (config 5's MFMA-bf16 mode, not bit-exact by construction), bounded against
      the same oracle output: max |conf - oracle| <= 2e-3 (measured 5.5e-4), matches0 equal on every row whose
      oracle score is > 0.5, and >= 99% of all rows equal."""
    from oracle import matcher_np as M
    n1, n3, L, seed = 2048, 8192, 8, 11
    sd = synthetic.make_state_dict(0)
    data, _, _ = synthetic.make_matcher_inputs(n1, n3, L, seed=seed, batch=1)
    opred, oconf = M.forward(sd, data)
    d2 = data["descriptors2d_query"]
    p32, c32 = CachedMatcher(sd, data, device, precision=0)(d2, with_conf=True)
    np.testing.assert_allclose(c32[0], oconf[0], rtol=0, atol=ATOL)
    assert_pred_equal(p32[0], opred, "config 5 fp32 vs oracle")
    om0, os0 = opred["matches0"].reshape(-1), opred["matching_scores0"].reshape(-1)
    assert (om0 > -1).sum() > 0.2 * n1
    p16, c16 = CachedMatcher(sd, data, device, precision=1)(d2, with_conf=True)
    dconf = float(np.abs(c16[0] - oconf[0]).max())
    m16 = p16[0]["matches0"]
    conf_rows = os0 > 0.5
    agree = float((m16 == om0).mean())
    print(f"config 5 bf16 vs oracle: max |dconf| {dconf:.3e}, rows equal {agree:.5f}, "
          f"confident rows {int(conf_rows.sum())} all equal: "
          f"{bool((m16[conf_rows] == om0[conf_rows]).all())}")
    assert dconf <= 2e-3
    assert (m16[conf_rows] == om0[conf_rows]).all()
    assert agree >= 0.99


def _fp16_rounded(data):
    """The matcher inputs with every descriptor rounded to fp16, as fp16 and upcast to fp32."""
    keys = ("descriptors2d_query", "descriptors3d_db", "descriptors2d_db")
    h = {k: (v.astype(np.float16) if k in keys else v) for k, v in data.items()}
    up = {k: (v.astype(np.float32) if k in keys else v) for k, v in h.items()}
    return h, up


@pytest.mark.parametrize("precision", [0, 1, 2])
def test_fp16_descriptors_equal_the_upcast_fp32_path(precision, device):
    """fp16 descriptors (BASELINE config 5's "fp16 desc"), converted by the kernels as they load
    them, give the bits of the fp32 path on the upcast inputs (GATs_SuperGlue.py:219-221 .float()):
    the cached path (object prepare + match_cached) and the module forward, every precision."""
    sd = synthetic.make_state_dict(0)
    data, _, _ = synthetic.make_matcher_inputs(300, 1000, 8, seed=4, batch=2)
    h, up = _fp16_rounded(data)
    p16, c16 = CachedMatcher(sd, data, device, precision=precision, fp16=True)(
        data["descriptors2d_query"], with_conf=True)
    p32, c32 = CachedMatcher(sd, up, device, precision=precision)(
        up["descriptors2d_query"], with_conf=True)
    np.testing.assert_array_equal(c16, c32)
    for a, b in zip(p16, p32):
        for k in a:
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    prec = {0: "fp32", 1: "bf16", 2: "fp32_split"}[precision]
    m = matcher.from_state_dict(sd, {**synthetic.DEFAULT_HPARAMS, "attention_precision": prec})
    m = m.to(device)
    with torch.no_grad():
        th = {k: torch.from_numpy(v).to(device) for k, v in h.items()}
        tu = {k: torch.from_numpy(v).to(device) for k, v in up.items()}
        assert th["descriptors2d_db"].dtype == torch.float16
        ph, ch = m(th)
        pu, cu = m(tu)
    np.testing.assert_array_equal(ch.cpu().numpy(), cu.cpu().numpy())
    for k in ph:
        np.testing.assert_array_equal(ph[k].cpu().numpy(), pu[k].cpu().numpy(), err_msg=k)


def test_config5_fp16_descriptors_vs_oracle(device):
    """BASELINE config 5 as named: 2048 x 8192, fp16 descriptors.  fp32 attention: indices
    exact and conf within 2e-5 against the numpy oracle on the upcast inputs; MFMA-bf16
    attention: bit-identical to the bf16 mode on the upcast fp32 inputs."""
    from oracle import matcher_np as M
    n1, n3, L, seed = 2048, 8192, 8, 11
    sd = synthetic.make_state_dict(0)
    data, _, _ = synthetic.make_matcher_inputs(n1, n3, L, seed=seed, batch=1)
    _, up = _fp16_rounded(data)
    opred, oconf = M.forward(sd, up)
    p16, c16 = CachedMatcher(sd, data, device, precision=0, fp16=True)(
        data["descriptors2d_query"], with_conf=True)
    np.testing.assert_allclose(c16[0], oconf[0], rtol=0, atol=ATOL)
    assert_pred_equal(p16[0], opred, "config 5 fp16 desc, fp32 vs oracle")
    b16, bc16 = CachedMatcher(sd, data, device, precision=1, fp16=True)(
        data["descriptors2d_query"], with_conf=True)
    b32, bc32 = CachedMatcher(sd, up, device, precision=1)(up["descriptors2d_query"], with_conf=True)
    np.testing.assert_array_equal(bc16, bc32)
    np.testing.assert_array_equal(b16[0]["matches0"], b32[0]["matches0"])
