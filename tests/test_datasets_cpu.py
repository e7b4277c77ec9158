"""Frame sources and checkpoint format on synthetic folders.

The reference's src/utils/datasets.py imports cv2 (absent here), so its classes cannot be run: the
checks restate its contract — file discovery and sort order (datasets.py:120-123, 186-189),
traj.txt / pose/*.txt / trajectory.log parsing with the y/z flip (:127-137, :152-178, :193-208),
depth / png_depth_scale × scale (:92,96), crop_edge (:106-110), translation × scale (:112) — and
the colour resize against a numpy restatement of cv2.resize INTER_LINEAR (half-pixel centres,
border clamp).  JPEG decoding is Pillow's on both sides (parity with cv2's decoder unpinned).
"""
import importlib
import os
from types import SimpleNamespace

import numpy as np
import pytest
import torch
from PIL import Image

P = importlib.import_module("nice-slam_amd")


def cv2_linear_resize(img, H, W):
    """cv2.resize(img, (W, H), INTER_LINEAR) for a float image: src = (dst+0.5)*in/out - 0.5,
    clamped at 0; the right neighbour clamped to the last pixel."""
    def axis(n_out, n_in):
        s = (np.arange(n_out) + 0.5) * (n_in / n_out) - 0.5
        s = np.maximum(s, 0.0)
        i0 = np.minimum(np.floor(s).astype(int), n_in - 1)
        i1 = np.minimum(i0 + 1, n_in - 1)
        return i0, i1, s - i0
    y0, y1, fy = axis(H, img.shape[0])
    x0, x1, fx = axis(W, img.shape[1])
    top = img[y0][:, x0] * (1 - fx)[None, :, None] + img[y0][:, x1] * fx[None, :, None]
    bot = img[y1][:, x0] * (1 - fx)[None, :, None] + img[y1][:, x1] * fx[None, :, None]
    return top * (1 - fy)[:, None, None] + bot * fy[:, None, None]


def _cfg(name, folder, H, W, depth_scale, crop_edge=0):
    return {"dataset": name, "data": {"input_folder": folder},
            "cam": {"H": H, "W": W, "fx": 100.0, "fy": 100.0, "cx": W / 2, "cy": H / 2,
                    "png_depth_scale": depth_scale, "crop_edge": crop_edge}}


def _poses(rng, n):
    return [rng.normal(size=(4, 4)) for _ in range(n)]


def _flipped(m, scale=1.0):
    m = m.copy()
    m[:3, 1] *= -1
    m[:3, 2] *= -1
    m[:3, 3] *= scale
    return m.astype(np.float32)


def test_replica_folder(tmp_path):
    rng = np.random.default_rng(0)
    H, W, n = 24, 32, 3
    os.makedirs(tmp_path / "results")
    deps = []
    for i in range(n):
        Image.fromarray(rng.integers(0, 256, (H, W, 3), dtype=np.uint8)).save(tmp_path / f"results/frame{i:06d}.jpg")
        d = rng.integers(0, 65535, (H, W)).astype(np.uint16)
        deps.append(d)
        Image.fromarray(d).save(tmp_path / f"results/depth{i:06d}.png")
    poses = _poses(rng, n)
    with open(tmp_path / "traj.txt", "w") as f:
        for m in poses:
            f.write(" ".join(f"{v:.17g}" for v in m.ravel()) + "\n")
    ds = P.get_dataset(_cfg("replica", str(tmp_path), H, W, 6553.5), None, 2.0, device="cpu")
    assert len(ds) == n
    for i in range(n):
        idx, color, depth, pose = ds[i]
        assert idx == i
        ref_c = np.asarray(Image.open(tmp_path / f"results/frame{i:06d}.jpg").convert("RGB")) / 255.0
        assert color.dtype == torch.float64 and np.array_equal(color.numpy(), ref_c)
        assert depth.dtype == torch.float32
        np.testing.assert_array_equal(depth.numpy(), (deps[i].astype(np.float32) / 6553.5) * 2.0)
        np.testing.assert_allclose(pose.numpy(), _flipped(poses[i], 2.0), rtol=1e-7)


def test_scannet_folder_resize_sort_and_crop(tmp_path):
    rng = np.random.default_rng(1)
    H, W, e = 24, 32, 2
    base = tmp_path / "frames"
    for sub in ("color", "depth", "pose"):
        os.makedirs(base / sub)
    stems = [10, 2, 0]  # integer sort → 0, 2, 10 (lexicographic would put 10 before 2)
    poses, deps = {}, {}
    for s in stems:
        Image.fromarray(rng.integers(0, 256, (37, 50, 3), dtype=np.uint8)).save(base / f"color/{s}.jpg")
        deps[s] = rng.integers(0, 8000, (H, W)).astype(np.uint16)
        Image.fromarray(deps[s]).save(base / f"depth/{s}.png")
        poses[s] = rng.normal(size=(4, 4))
        with open(base / f"pose/{s}.txt", "w") as f:
            f.write("\n".join(" ".join(f"{v:.17g}" for v in row) for row in poses[s]) + "\n")
    ds = P.get_dataset(_cfg("scannet", str(tmp_path), H, W, 1000.0, crop_edge=e), None, 1.0, device="cpu")
    assert [os.path.basename(p) for p in ds.color_paths] == ["0.jpg", "2.jpg", "10.jpg"]
    for k, s in enumerate(sorted(stems)):
        _, color, depth, pose = ds[k]
        raw = np.asarray(Image.open(base / f"color/{s}.jpg").convert("RGB")) / 255.0
        ref = cv2_linear_resize(raw, H, W)[e:-e, e:-e]
        assert color.shape == (H - 2 * e, W - 2 * e, 3)
        np.testing.assert_allclose(color.numpy(), ref, atol=1e-6)
        np.testing.assert_array_equal(depth.numpy(), (deps[s].astype(np.float32) / 1000.0)[e:-e, e:-e])
        np.testing.assert_array_equal(pose.numpy(), _flipped(poses[s]))


def test_azure_trajectory_log(tmp_path):
    rng = np.random.default_rng(2)
    H, W, n = 16, 20, 2
    for sub in ("color", "depth", "scene"):
        os.makedirs(tmp_path / sub)
    poses = _poses(rng, n)
    with open(tmp_path / "scene/trajectory.log", "w") as f:
        for i, m in enumerate(poses):
            f.write(f"{i} {i} {i + 1}\n")
            for row in m:
                f.write(" ".join(f"{v:.17g}" for v in row) + "\n")
    for i in range(n):
        Image.fromarray(rng.integers(0, 256, (H, W, 3), dtype=np.uint8)).save(tmp_path / f"color/{i:05d}.jpg")
        Image.fromarray(rng.integers(0, 9000, (H, W)).astype(np.uint16)).save(tmp_path / f"depth/{i:05d}.png")
    ds = P.get_dataset(_cfg("azure", str(tmp_path), H, W, 1000.0), SimpleNamespace(input_folder=None), 1.0,
                       device="cpu", color_dtype=torch.float32)
    for i in range(n):
        _, color, _, pose = ds[i]
        assert color.dtype == torch.float32
        np.testing.assert_array_equal(pose.numpy(), _flipped(poses[i]))


def test_unsupported_dataset_raises():
    with pytest.raises(NotImplementedError):
        P.get_dataset({"dataset": "cofusion"}, None, 1.0, device="cpu")


def test_checkpoint_roundtrip(tmp_path):
    nice = P.NICE(c_dim=32, coarse=True)
    grids = {k: torch.randn(1, 32, 3, 4, 5).contiguous(memory_format=torch.channels_last_3d)
             for k in ("grid_coarse", "grid_middle", "grid_fine", "grid_color")}
    gt, est = torch.randn(4, 4, 4), torch.randn(4, 4, 4)
    path = str(tmp_path / "00003.tar")
    P.datasets.save_checkpoint(path, grids, nice, gt, est, [0, 2], 3)
    ck = P.datasets.load_checkpoint(path, device="cpu")
    assert set(ck) == {"c", "decoder_state_dict", "gt_c2w_list", "estimate_c2w_list", "keyframe_list",
                       "selected_keyframes", "idx"}
    for k, v in grids.items():
        assert ck["c"][k].is_contiguous(memory_format=torch.channels_last_3d) and torch.equal(ck["c"][k], v)
    sd = nice.state_dict()
    assert list(ck["decoder_state_dict"]) == list(sd)
    assert all(torch.equal(ck["decoder_state_dict"][k], sd[k]) for k in sd)
    assert torch.equal(ck["estimate_c2w_list"], est) and ck["keyframe_list"] == [0, 2] and ck["idx"] == 3


@pytest.mark.gpu
def test_device_frames_equal_host_frames(tmp_path):
    """On the device the /255, /png_depth_scale, resize and crops run after the uint8/float32 upload:
    depth and pose equal the host computation bit for bit; colour to 1e-12 (the resize kernel's
    rounding may differ between the CPU and GPU interpolate implementations)."""
    test_scannet_folder_resize_sort_and_crop(tmp_path)  # writes the folder
    cfg = _cfg("scannet", str(tmp_path), 24, 32, 1000.0, crop_edge=2)
    host = P.get_dataset(cfg, None, 1.0, device="cpu")
    dev = P.get_dataset(cfg, None, 1.0, device="cuda:0")
    for k in range(len(host)):
        _, c0, d0, p0 = host[k]
        _, c1, d1, p1 = dev[k]
        assert c1.is_cuda and torch.allclose(c1.cpu(), c0, rtol=0, atol=1e-12) and torch.equal(d1.cpu(), d0) and torch.equal(p1.cpu(), p0)


def _prefetch_equals_getitem(tmp_path, device):
    test_scannet_folder_resize_sort_and_crop(tmp_path)  # writes the folder
    cfg = _cfg("scannet", str(tmp_path), 24, 32, 1000.0, crop_edge=2)
    a = P.get_dataset(cfg, None, 0.5, device=device)
    b = P.get_dataset(cfg, None, 0.5, device=device)
    order = [2, 0, 1]
    got = list(a.prefetch(order, workers=2, ahead=3))
    assert [g[0] for g in got] == order
    for g in got:
        e = b[g[0]]
        assert g[1].device == e[1].device
        for x, y in zip(g[1:], e[1:]):
            assert x.dtype == y.dtype and torch.equal(x.cpu(), y.cpu())


def test_prefetch_yields_getitem(tmp_path):
    """BaseDataset.prefetch (the reference's DataLoader worker, Tracker.py:64-65): decode in worker
    processes, then the same device half as __getitem__ — the same tuples, in the requested order."""
    _prefetch_equals_getitem(tmp_path, "cpu")


@pytest.mark.gpu
def test_prefetch_yields_getitem_on_device(tmp_path):
    """The same on the GPU: pinned host buffers, H2D + normalisation on a side stream."""
    _prefetch_equals_getitem(tmp_path, "cuda:0")
