"""The inference.py-compatible driver's host side (onepose_amd/inference.py): path rules of
path_utils.py, the on-disk object format, safe checkpoint loading, image normalisation."""
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
    imgs, paths = I.get_default_paths(str(seq), str(tmp_path / "sfm"))
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
