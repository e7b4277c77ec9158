"""Golden vectors for the frame and checkpoint formats, produced by the
reference's own code (build container only; the .npz it writes is what tests/test_io_golden.py reads).

Run:  PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_io.py

Cases (reference file:line they execute):
  replica   src/utils/datasets.py Replica (:116-137) + BaseDataset.__getitem__ (:77-113) on a
            synthetic results/frame*.jpg + depth*.png + traj.txt folder, scale 1.5, crop_edge 2.
  scannet   ScanNet (:181-208): frames/color/<n>.jpg larger than frames/depth/<n>.png (the colour
            resize, :94), numeric sort of the stems (1, 2, 10), pose/<n>.txt, crop_size (:97-104),
            crop_edge 1.
  azure     Azure (:140-178): color/*.jpg, depth/*.png, scene/trajectory.log (5-line records).
  ckpt      src/utils/Logger.py Logger.log (:21-32): the legacy-serialised checkpoint dict of a
            reference NICE (decoder.py) with its shared grids, pose lists and keyframe list.

Harness (nothing of the reference is copied or modified; it is imported and called):
  * src.utils.datasets imports cv2 (absent).  A stand-in module is registered first with the four
    calls __getitem__ makes: imread (Pillow decode, BGR channel order like OpenCV; 16-bit PNG as
    uint16 for IMREAD_UNCHANGED), cvtColor(BGR2RGB) (channel reversal) and resize INTER_LINEAR (a
    numpy restatement: half-pixel centres, edge clamp, float64).  The fixtures therefore pin the
    reference's code AROUND those calls — file discovery and sort order, pose parsing and the y/z
    flip, /255 and png_depth_scale, scale, crop_size, crop_edge, the in-place pose scaling — while
    parity of the decode and resample with OpenCV itself stays unpinned (library absent).
  * The input files (JPEG / PNG / text bytes) are stored in the .npz, so the test rebuilds exactly
    the folders the reference read.
"""
import io
import os
import sys
import tempfile
import types
from types import SimpleNamespace

import numpy as np
import torch
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)


def linear_resize(img, W, H):
    """cv2.resize(img, (W, H), interpolation=INTER_LINEAR) for a float image: src = (dst + 0.5) ·
    in / out − 0.5 clamped at 0, the upper neighbour clamped to the last pixel."""
    img = np.asarray(img, dtype=np.float64)

    def axis(n_out, n_in):
        s = (np.arange(n_out) + 0.5) * (n_in / n_out) - 0.5
        s = np.maximum(s, 0.0)
        i0 = np.minimum(np.floor(s).astype(np.int64), n_in - 1)
        i1 = np.minimum(i0 + 1, n_in - 1)
        return i0, i1, s - i0

    if img.shape[0] == H and img.shape[1] == W:
        return img.copy()
    y0, y1, fy = axis(H, img.shape[0])
    x0, x1, fx = axis(W, img.shape[1])
    top = img[y0][:, x0] * (1 - fx)[None, :, None] + img[y0][:, x1] * fx[None, :, None]
    bot = img[y1][:, x0] * (1 - fx)[None, :, None] + img[y1][:, x1] * fx[None, :, None]
    return top * (1 - fy)[:, None, None] + bot * fy[:, None, None]


def install_cv2():
    cv2 = types.ModuleType("cv2")
    cv2.IMREAD_UNCHANGED = -1
    cv2.COLOR_BGR2RGB = 4
    cv2.INTER_LINEAR = 1

    def imread(path, flags=1):
        with Image.open(path) as im:
            if flags == cv2.IMREAD_UNCHANGED:
                return np.asarray(im).copy()
            return np.asarray(im.convert("RGB"))[..., ::-1].copy()  # OpenCV's BGR order

    def cvtColor(img, code):
        assert code == cv2.COLOR_BGR2RGB
        return img[..., ::-1].copy()

    def resize(img, dsize, interpolation=1):
        return linear_resize(img, dsize[0], dsize[1])

    cv2.imread, cv2.cvtColor, cv2.resize = imread, cvtColor, resize
    sys.modules["cv2"] = cv2


def jpeg_bytes(arr):
    b = io.BytesIO()
    Image.fromarray(arr).save(b, format="JPEG", quality=92)
    return b.getvalue()


def png16_bytes(arr):
    b = io.BytesIO()
    Image.fromarray(arr.astype(np.uint16)).save(b, format="PNG")
    return b.getvalue()


def smooth_image(rng, H, W):
    yy, xx = np.mgrid[0:H, 0:W]
    ph = rng.uniform(0, 6, 3)
    img = np.stack([127 + 120 * np.sin(xx / (3 + k) + yy / (5 + k) + ph[k]) for k in range(3)], -1)
    return np.clip(img, 0, 255).astype(np.uint8)


def pose_text(m):
    return " ".join(repr(float(v)) for v in m.ravel())


def write_files(root, files):
    for rel, data in files.items():
        p = os.path.join(root, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "wb") as f:
            f.write(data)


def dataset_case(out, name, cls, files, cfg, scale):
    with tempfile.TemporaryDirectory() as d:
        write_files(d, files)
        cfg = dict(cfg, dataset=name, data={"input_folder": d})
        ds = cls(cfg, SimpleNamespace(input_folder=None), scale, device="cpu")
        out[f"{name}.n"] = np.array(len(ds))
        for i in range(len(ds)):
            idx, color, depth, pose = ds[i]
            out[f"{name}.{i}.index"] = np.array(idx)
            out[f"{name}.{i}.color"] = color.numpy()
            out[f"{name}.{i}.depth"] = depth.numpy()
            out[f"{name}.{i}.pose"] = pose.numpy()
    names = sorted(files)
    out[f"{name}.files"] = np.array(names)
    for k, rel in enumerate(names):
        out[f"{name}.file{k}"] = np.frombuffer(files[rel], dtype=np.uint8)
    out[f"{name}.scale"] = np.array(scale)
    for k, v in cfg["cam"].items():
        out[f"{name}.cam.{k}"] = np.array(v)


def main():
    install_cv2()
    from src.conv_onet.models.decoder import NICE  # noqa: E402  (reference)
    from src.utils import datasets as R  # noqa: E402  (reference)
    from src.utils.Logger import Logger  # noqa: E402  (reference)

    rng = np.random.default_rng(4)
    out = {}
    cam = {"H": 24, "W": 32, "fx": 30.0, "fy": 31.0, "cx": 15.5, "cy": 11.5, "png_depth_scale": 6553.5}

    # Replica: results/frame*.jpg, results/depth*.png, traj.txt
    files = {}
    traj = []
    for i in range(3):
        files[f"results/frame{i:06d}.jpg"] = jpeg_bytes(smooth_image(rng, 24, 32))
        files[f"results/depth{i:06d}.png"] = png16_bytes(rng.integers(0, 40000, (24, 32)))
        traj.append(pose_text(rng.normal(size=(4, 4))))
    files["traj.txt"] = ("\n".join(traj) + "\n").encode()
    dataset_case(out, "replica", R.Replica, files, {"cam": dict(cam, crop_edge=2)}, 1.5)

    # ScanNet: colour larger than depth (resize), numeric stem order, pose/<n>.txt, crop_size
    files = {}
    for i in (1, 2, 10):
        files[f"frames/color/{i}.jpg"] = jpeg_bytes(smooth_image(rng, 30, 40))
        files[f"frames/depth/{i}.png"] = png16_bytes(rng.integers(0, 5000, (24, 32)))
        m = rng.normal(size=(4, 4))
        files[f"frames/pose/{i}.txt"] = ("\n".join(" ".join(repr(float(v)) for v in row) for row in m) + "\n").encode()
    dataset_case(out, "scannet", R.ScanNet, files,
                 {"cam": dict(cam, png_depth_scale=1000.0, crop_edge=1, crop_size=[20, 28])}, 1.0)

    # Azure (Apartment): color/*.jpg, depth/*.png, scene/trajectory.log
    files = {}
    log = []
    for i in range(2):
        files[f"color/{i:05d}.jpg"] = jpeg_bytes(smooth_image(rng, 24, 32))
        files[f"depth/{i:05d}.png"] = png16_bytes(rng.integers(0, 3000, (24, 32)))
        m = rng.normal(size=(4, 4))
        log.append(f"{i} {i} 0.0")
        log += [" ".join(repr(float(v)) for v in row) for row in m]
    files["scene/trajectory.log"] = ("\n".join(log) + "\n").encode()
    dataset_case(out, "azure", R.Azure, files, {"cam": dict(cam, png_depth_scale=1000.0, crop_edge=0)}, 1.0)

    # Logger.log: the checkpoint dict, legacy serialisation
    torch.manual_seed(5)
    nice = NICE(dim=3, c_dim=32, coarse_grid_len=2.0, middle_grid_len=0.64, fine_grid_len=0.32, color_grid_len=0.32,
                hidden_size=32, coarse=True, pos_embedding_method="fourier")
    shapes = {"grid_coarse": (1, 32, 2, 3, 2), "grid_middle": (1, 32, 4, 5, 6), "grid_fine": (1, 32, 8, 9, 10),
              "grid_color": (1, 32, 8, 9, 10)}
    shared_c = {k: torch.randn(s) * 0.01 for k, s in shapes.items()}
    gt = torch.randn(6, 4, 4)
    est = torch.randn(6, 4, 4)
    with tempfile.TemporaryDirectory() as d:
        slam = SimpleNamespace(verbose=False, ckptsdir=d, shared_c=shared_c, gt_c2w_list=gt, shared_decoders=nice,
                               estimate_c2w_list=est)
        Logger(None, None, slam).log(5, {}, [0, 2, 4], selected_keyframes=[2, 4])
        with open(os.path.join(d, "00005.tar"), "rb") as f:
            out["ckpt.tar"] = np.frombuffer(f.read(), dtype=np.uint8)
    for k, v in shared_c.items():
        out["ckpt.c." + k] = v.numpy()
    for k, v in nice.state_dict().items():
        out["ckpt.sd." + k] = v.numpy()
    out["ckpt.gt_c2w_list"] = gt.numpy()
    out["ckpt.estimate_c2w_list"] = est.numpy()
    path = os.path.join(HERE, "io_fixtures.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(out)} arrays, {os.path.getsize(path) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
