"""Frame and checkpoint formats against the reference's own outputs.

tests/golden/io_fixtures.npz was written by tests/golden/make_golden_io.py, which ran the
reference's src/utils/datasets.py (Replica, ScanNet, Azure: BaseDataset.__getitem__ with a stand-in
cv2 — Pillow decode, a numpy INTER_LINEAR resize) and src/utils/Logger.py (Logger.log) in the build
container.  The input files are stored in the fixture, so the product's loaders read exactly the
folders the reference read.  Pinned to the reference: file discovery and sort order, pose parsing
and the y/z flip, /255 and png_depth_scale, scale, crop_size, crop_edge, the checkpoint dict and its
legacy serialisation.  Unpinned (cv2 absent): OpenCV's own JPEG decoder and resampler.
"""
import importlib
import os

import numpy as np
import pytest
import torch

P = importlib.import_module("nice-slam_amd")
FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "io_fixtures.npz")


@pytest.fixture(scope="module")
def fx():
    with np.load(FIX) as z:
        return {k: z[k] for k in z.files}


def _rebuild(fx, name, root):
    for k, rel in enumerate(fx[f"{name}.files"]):
        p = os.path.join(root, str(rel))
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "wb") as f:
            f.write(fx[f"{name}.file{k}"].tobytes())
    cam = {}
    for key in fx:
        if key.startswith(f"{name}.cam."):
            v = fx[key]
            cam[key[len(name) + 5:]] = v.tolist() if v.ndim else v.item()
    return {"dataset": name, "data": {"input_folder": str(root)}, "cam": cam}


@pytest.mark.parametrize("name", ["replica", "scannet", "azure"])
def test_dataset_matches_reference(fx, tmp_path, name):
    cfg = _rebuild(fx, name, tmp_path)
    ds = P.get_dataset(cfg, None, float(fx[f"{name}.scale"]), device="cpu")
    assert len(ds) == int(fx[f"{name}.n"])
    for i in range(len(ds)):
        idx, color, depth, pose = ds[i]
        assert idx == int(fx[f"{name}.{i}.index"])
        ref_c, ref_d, ref_p = fx[f"{name}.{i}.color"], fx[f"{name}.{i}.depth"], fx[f"{name}.{i}.pose"]
        assert color.dtype == torch.float64 and tuple(color.shape) == ref_c.shape
        assert depth.dtype == torch.float32 and tuple(depth.shape) == ref_d.shape
        # depth, pose: the same float operations as the reference — bit-exact
        assert np.array_equal(depth.numpy(), ref_d), (name, i)
        assert np.array_equal(pose.numpy(), ref_p), (name, i)
        # colour: bit-exact when no resize runs; the resize (torch bilinear vs the fixture's numpy
        # INTER_LINEAR restatement, both float64) to rounding
        err = float(np.abs(color.numpy() - ref_c).max())
        assert err < 1e-12, (name, i, err)


def test_checkpoint_written_by_reference_loads(fx, tmp_path):
    """Logger.log's .tar (legacy serialisation) through the product's load_checkpoint
    (weights_only=True): every key and value, grids back channels-last, the decoder state_dict into
    the product's NICE (same keys, strict)."""
    path = tmp_path / "00005.tar"
    path.write_bytes(fx["ckpt.tar"].tobytes())
    ck = P.datasets.load_checkpoint(str(path), device="cpu")
    assert set(ck) == {"c", "decoder_state_dict", "gt_c2w_list", "estimate_c2w_list", "keyframe_list",
                       "selected_keyframes", "idx"}
    assert ck["idx"] == 5 and ck["keyframe_list"] == [0, 2, 4] and ck["selected_keyframes"] == [2, 4]
    for k, g in ck["c"].items():
        assert g.is_contiguous(memory_format=torch.channels_last_3d), k
        assert np.array_equal(g.numpy(), fx["ckpt.c." + k]), k
    assert np.array_equal(ck["gt_c2w_list"].numpy(), fx["ckpt.gt_c2w_list"])
    assert np.array_equal(ck["estimate_c2w_list"].numpy(), fx["ckpt.estimate_c2w_list"])
    sd = ck["decoder_state_dict"]
    assert set(sd) == {k[len("ckpt.sd."):] for k in fx if k.startswith("ckpt.sd.")}
    nice = P.NICE(c_dim=32, coarse_grid_len=2.0, middle_grid_len=0.64, fine_grid_len=0.32, color_grid_len=0.32,
                  hidden_size=32, coarse=True)
    nice.load_state_dict(sd)  # strict: the product's module has the reference's parameter names
    for k, v in nice.state_dict().items():
        assert np.array_equal(v.numpy(), fx["ckpt.sd." + k]), k


def test_checkpoint_written_by_product_equals_reference(fx, tmp_path):
    """save_checkpoint of the same content == the reference's file, entry by entry, as the
    reference's consumers (NICE_SLAM / Mesher: torch.load) see it."""
    ref = tmp_path / "ref.tar"
    ref.write_bytes(fx["ckpt.tar"].tobytes())
    a = torch.load(str(ref), map_location="cpu", weights_only=True)
    nice = P.NICE(c_dim=32, coarse_grid_len=2.0, middle_grid_len=0.64, fine_grid_len=0.32, color_grid_len=0.32,
                  hidden_size=32, coarse=True)
    nice.load_state_dict(a["decoder_state_dict"])
    ours = tmp_path / "ours.tar"
    P.datasets.save_checkpoint(str(ours), a["c"], nice, a["gt_c2w_list"], a["estimate_c2w_list"], a["keyframe_list"],
                               a["idx"], selected_keyframes=a["selected_keyframes"])
    with open(ours, "rb") as f:
        assert f.read(2) != b"PK"  # legacy (non-zip) serialisation, like Logger.py:32
    b = torch.load(str(ours), map_location="cpu", weights_only=True)
    assert list(a) == list(b)
    for k in a:
        if k == "c" or k == "decoder_state_dict":
            assert list(a[k]) == list(b[k]), k
            for kk in a[k]:
                assert torch.equal(a[k][kk], b[k][kk]), (k, kk)
        elif torch.is_tensor(a[k]):
            assert torch.equal(a[k], b[k]), k
        else:
            assert a[k] == b[k], k
