"""The inference.py-compatible driver's host side (onepose_amd/inference.py): path rules of
path_utils.py, the on-disk object format, safe checkpoint loading, image normalisation, and
the reference entry chain's host pieces (get_default_paths(cfg, ...), LitModelGATsSPG,
NormalizedDataset batches, record_eval_result against the reference's own output)."""
import os

import numpy as np
import pytest
import torch

from onepose_amd import inference as I
from onepose_amd import synthetic as S


def test_path_rules_both_separators():
    for sep in ("/", "\\"):
        p = sep.join(["", "data", "obj", "seq-1", "color", "12.png"])
        assert I.get_intrin_path_by_color(p) == sep.join(["", "data", "obj", "seq-1", "intrin_ba", "12.txt"])
        assert I.get_gt_pose_path_by_color(p) == sep.join(["", "data", "obj", "seq-1", "poses_ba", "12.txt"])
        q = p.replace("color", "color_det")
        assert I.get_intrin_path_by_color(q, "feature_matching").endswith(
            sep.join(["intrin_det", "12.txt"]))
        assert I.get_gt_pose_path_by_color(q, "feature_matching").endswith(
            sep.join(["poses_ba", "12.txt"]))
    with pytest.raises(NotImplementedError):
        I.get_intrin_path_by_color("/a/color/1.png", "other")


def test_default_paths_and_object_roundtrip(tmp_path):
    seq = tmp_path / "seq"
    (seq / "color").mkdir(parents=True)
    for i in (3, 1, 2):
        (seq / "color" / f"{i}.png").write_bytes(b"")
    imgs, paths = I.default_paths(str(seq), str(tmp_path / "sfm"))
    assert [os.path.basename(p) for p in imgs] == ["1.png", "2.png", "3.png"]
    assert paths["anno_dir"].endswith(os.path.join("outputs_superpoint_superglue", "anno"))
    obj = S.make_object(50, seed=3)
    from onepose_amd import data_utils as DU
    DU.save_object_annotations(paths["anno_dir"], obj.keypoints3d, obj.clt_descriptors,
                               obj.clt_scores, obj.idxs)
    I.seed_reference_stream()
    o = I.OnePoseObject.from_anno_dir(paths["anno_dir"], 8, device="cpu")
    assert o.keypoints3d.shape == (50, 3) and o.descriptors3d.shape == (256, 50)
    assert o.leaves.shape == (256, 400) and o.num_leaf == 8
    np.testing.assert_allclose(o.descriptors3d.numpy(), obj.avg_descriptors, rtol=1e-5, atol=1e-6)


def test_lightning_checkpoint_loads_safely(tmp_path):
    sd = S.make_state_dict(0)
    ckpt = {"state_dict": {"matcher." + k: torch.from_numpy(v) for k, v in sd.items()},
            "hyper_parameters": {"match_threshold": 0.3, "scale_factor": 0.07,
                                 "match_type": "softmax"}}
    ckpt["state_dict"]["extractor.conv1a.weight"] = torch.zeros(1)   # ignored
    path = tmp_path / "GATsSPG.ckpt"
    torch.save(ckpt, path)
    m = I.load_matcher(str(path))
    assert m.hparams["match_threshold"] == 0.3
    got = m.state_dict()
    for k in ("gnn.layers.1.attn.proj.0.weight", "final_proj.bias"):
        np.testing.assert_array_equal(got[k].numpy(), sd[k])


def test_load_image_grayscale_normalisation(tmp_path):
    from PIL import Image
    a = (np.arange(64 * 48) % 256).astype(np.uint8).reshape(48, 64)
    Image.fromarray(a, mode="L").save(tmp_path / "x.png")
    img, size = I.load_image(str(tmp_path / "x.png"))
    assert img.shape == (1, 48, 64) and tuple(size) == (48, 64) and img.dtype == np.float32
    np.testing.assert_array_equal(img[0], a.astype(np.float32) / 255.0)


def _cfg(**kw):
    from types import SimpleNamespace as N
    base = dict(network=N(detection="superpoint", matching="superglue"),
                object_detect_mode="GT_box", num_leaf=8)
    base.update(kw)
    return N(**base)


def test_get_default_paths_reference_signature(tmp_path):
    """inference.py:17-46: get_default_paths(cfg, data_root, data_dir, sfm_model_dir)."""
    seq = tmp_path / "root" / "seq-1"
    (seq / "color").mkdir(parents=True)
    (seq / "color" / "0.png").write_bytes(b"")
    imgs, paths = I.get_default_paths(_cfg(), str(tmp_path / "root"), str(seq),
                                      str(tmp_path / "sfm" / "obj"))
    assert imgs == [str(seq / "color" / "0.png")]
    assert paths["data_root"] == str(tmp_path / "root") and paths["data_dir"] == str(seq)
    assert paths["avg_anno_3d_path"] == os.path.join(
        str(tmp_path / "sfm" / "obj"), "outputs_superpoint_superglue", "anno", "anno_3d_average.npz")
    assert paths["intrin_full_path"] == os.path.join(str(seq), "intrinsics.txt")
    with pytest.raises(FileNotFoundError):   # the reference asserts color_det exists
        I.get_default_paths(_cfg(object_detect_mode="feature_matching"), "", str(seq), "")
    with pytest.raises(NotImplementedError):
        I.get_default_paths(_cfg(object_detect_mode="other"), "", str(seq), "")


def test_record_eval_result_matches_reference(tmp_path):
    """eval_utils.py:7-15: the file the reference wrote for the same summary (golden)."""
    from onepose_amd import pose
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "eval_record.npz"))
    ev = pose.Evaluator()
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "evaluator.npz"))
    for p, gt in zip(g["preds"], g["gts"]):
        ev.evaluate(p, gt)
    summ = ev.summarize()
    out_dir = tmp_path / "runs" / "eval" / "GATsSPG"
    path = pose.record_eval_result(str(out_dir), "0408-colorbox-box", "colorbox-4", summ)
    assert os.listdir(out_dir) == [str(z["names"][0])]
    assert open(path).read() == str(z["text"])


def test_lightning_model_checkpoint_surface(tmp_path):
    """GATsSPG_lightning_model.py:15-37 + inference.py:55-58 on CPU: load_from_checkpoint,
    forward -> matcher, freeze."""
    from onepose_amd.lightning_model import LitModelGATsSPG
    sd = S.make_state_dict(1)
    ckpt = {"state_dict": {"matcher." + k: torch.from_numpy(v) for k, v in sd.items()},
            "hyper_parameters": {"match_threshold": 0.25, "scale_factor": 0.07,
                                 "match_type": "softmax", "focal_loss_alpha": 0.5}}
    ckpt["state_dict"]["crit.weight"] = torch.zeros(1)
    path = tmp_path / "GATsSPG.ckpt"
    torch.save(ckpt, path)
    m = LitModelGATsSPG.load_from_checkpoint(checkpoint_path=str(path))
    m.eval()
    m.freeze()
    assert m.matcher.hparams["match_threshold"] == 0.25
    assert not any(p.requires_grad for p in m.parameters())
    got = m.matcher.state_dict()
    np.testing.assert_array_equal(got["gnn.layers.4.mlp.0.weight"].numpy(),
                                  sd["gnn.layers.4.mlp.0.weight"])
    # forward is the matcher's: its empty-input path needs no GPU (GATs_SuperGlue.py:223-231)
    out = m({"keypoints2d": torch.zeros(1, 0, 2), "keypoints3d": torch.zeros(1, 5, 3)})
    assert out["skip_train"] and out["matches1"].tolist() == [-1] * 5


def test_normalized_dataset_batches(tmp_path):
    """normalized_dataset.py:22-41 collated by DataLoader(batch_size=1)."""
    from PIL import Image
    a = (np.arange(40 * 24) % 251).astype(np.uint8).reshape(24, 40)
    Image.fromarray(a, mode="L").save(tmp_path / "0.png")
    from onepose_amd.superpoint import confs
    ds = I.NormalizedDataset([str(tmp_path / "0.png")], confs["superpoint"]["preprocessing"])
    (b,) = list(ds.batches())
    assert b["path"] == [str(tmp_path / "0.png")]
    assert tuple(b["image"].shape) == (1, 1, 24, 40) and b["size"].tolist() == [[24, 40]]
    np.testing.assert_array_equal(b["image"][0, 0].numpy(), a.astype(np.float32) / 255.0)
    with pytest.raises(ValueError):
        I.NormalizedDataset([], {})
    # several images: read ahead by the worker, yielded in order; a bad file raises at its item;
    # a consumer that stops early does not leave the worker behind
    for i in (1, 2, 3):
        Image.fromarray((a + i).astype(np.uint8), mode="L").save(tmp_path / f"{i}.png")
    files = [str(tmp_path / f"{i}.png") for i in range(4)]
    ds = I.NormalizedDataset(files, confs["superpoint"]["preprocessing"])
    got = [b["path"][0] for b in ds.batches()]
    assert got == files
    bad = I.NormalizedDataset(files[:2] + [str(tmp_path / "missing.png")], {})
    it = bad.batches()
    assert next(it)["path"] == [files[0]] and next(it)["path"] == [files[1]]
    with pytest.raises(Exception):
        next(it)
    it = ds.batches()
    next(it)
    it.close()


def test_extractor_conf_threshold_typo():
    """extract_features.py:19-24 spells 'keypoints_threshold'; SuperPoint reads
    'keypoint_threshold', so the 0.005 default applies."""
    from onepose_amd.superpoint import SuperPoint, confs
    c = SuperPoint(confs["superpoint"]["conf"]).config
    assert c["keypoint_threshold"] == 0.005 and c["nms_radius"] == 3 and c["max_keypoints"] == 4096
