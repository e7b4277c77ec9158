"""Frame sources of the mapping/tracking path: Replica, ScanNet and Azure (Apartment) folders
(src/utils/datasets.py), plus the checkpoint dict of src/utils/Logger.py.

SURVEY.md §8(f) row 4.  Same classes, constructor arguments, sort orders and `__getitem__` contract
as the reference: `(index, color [H,W,3] float64 in [0,1], depth [H,W] float32 metres × scale,
c2w [4,4] float32 with the y/z axes flipped)`, on `device`.  Decoding uses Pillow (cv2 is not in
this image): JPEG/PNG pixels are Pillow's, the colour resize (datasets.py:94, cv2.resize INTER_LINEAR)
is restated as torch bilinear with half-pixel centres and border clamp — parity with cv2's own
decoder and resampler is unpinned (library absent); the pose parsing, axis flips, depth scaling,
crop_size interpolation and crop_edge are exact restatements.

`color_dtype=torch.float32` keeps a frame at half the bytes on the device (the fused engine reads
f32); the default float64 is the reference's (datasets.py:91).

`BaseDataset.prefetch(indices)` is the reference's DataLoader worker (Tracker.py:64-65, Mapper.py:
frame_reader): worker processes decode ahead into pinned host memory and each frame's H2D copy and
device-side normalisation run on a side stream, so decode overlaps the consumer's GPU work; it
yields exactly what `dataset[i]` returns (the same host half and device half).
Out of scope: CoFusion (OpenEXR), TUM-RGBD, lens undistortion (cv2.undistort) — none is a BASELINE
config; a config asking for `distortion` raises.
"""
from __future__ import annotations

import collections
import glob
import os

import numpy as np
import torch
import torch.nn.functional as F


def _read_color(path):
    from PIL import Image
    with Image.open(path) as im:
        return np.array(im.convert("RGB"))  # == cv2.imread + COLOR_BGR2RGB (datasets.py:80,90); writable


def _read_depth(path):
    from PIL import Image
    with Image.open(path) as im:  # 16-bit PNG → uint16 (cv2.IMREAD_UNCHANGED, datasets.py:82)
        return np.asarray(im)


def _flip_yz(c2w):
    """datasets.py:134-135 (and :170-171, :205-206): camera y and z axes negated."""
    c2w = np.array(c2w, dtype=np.float64).reshape(4, 4)
    c2w[:3, 1] *= -1
    c2w[:3, 2] *= -1
    return torch.from_numpy(c2w).float()


class BaseDataset(torch.utils.data.Dataset):
    """src/utils/datasets.py:51-113."""

    def __init__(self, cfg, args, scale, device="cuda:0", color_dtype=torch.float64):
        super().__init__()
        self.name = cfg["dataset"]
        self.device = device
        self.scale = scale
        self.color_dtype = color_dtype
        cam = cfg["cam"]
        self.png_depth_scale = cam["png_depth_scale"]
        self.H, self.W, self.fx, self.fy, self.cx, self.cy = cam["H"], cam["W"], cam["fx"], cam["fy"], cam["cx"], cam["cy"]
        if "distortion" in cam:
            raise NotImplementedError("lens undistortion (cv2.undistort) is out of scope")
        self.crop_size = cam.get("crop_size")
        folder = getattr(args, "input_folder", None) if args is not None else None
        self.input_folder = cfg["data"]["input_folder"] if folder is None else folder
        self.crop_edge = cam["crop_edge"]

    def __len__(self):
        return self.n_img

    def _lut(self, device):
        lut = getattr(self, "_u8_lut", None)
        if lut is None or lut.device != device:
            lut = self._u8_lut = (torch.arange(256, dtype=torch.float64) / 255.0).to(device)
        return lut

    def _load_host(self, index):
        """The host half of __getitem__: decoded colour bytes (uint8 [H,W,3]) and depth in metres
        before scaling (float32 [H,W]) — the part a prefetch worker process runs."""
        u8 = torch.from_numpy(np.ascontiguousarray(_read_color(self.color_paths[index])))
        depth = torch.from_numpy(_read_depth(self.depth_paths[index]).astype(np.float32) / np.float32(self.png_depth_scale))
        return u8, depth

    def __getitem__(self, index):
        return self._finish(index, *self._load_host(index))

    def _finish(self, index, u8, depth, non_blocking=False):
        # Only the decoded bytes cross PCIe for colour (uint8: 1/8 of the reference's float64 copy).
        # /255 (float64, datasets.py:91) is a 256-entry table divided on the host and gathered on
        # the device — torch's device kernels turn a scalar division into a reciprocal multiply,
        # which is not the reference's correctly-rounded quotient.  Depth is divided on the host
        # (float32, :92) for the same reason.  Resize and crops then run on the device.
        u8 = u8.to(self.device, non_blocking=non_blocking)
        color = self._lut(u8.device)[u8.long()]
        depth = depth.to(self.device, non_blocking=non_blocking)
        H, W = depth.shape
        if color.shape[:2] != (H, W):  # cv2.resize(color, (W, H)) INTER_LINEAR (datasets.py:94)
            color = F.interpolate(color.permute(2, 0, 1)[None], (H, W), mode="bilinear",
                                  align_corners=False)[0].permute(1, 2, 0)
        depth = depth * self.scale
        if self.crop_size is not None:  # datasets.py:97-104
            color = F.interpolate(color.permute(2, 0, 1)[None], self.crop_size, mode="bilinear",
                                  align_corners=True)[0].permute(1, 2, 0).contiguous()
            depth = F.interpolate(depth[None, None], self.crop_size, mode="nearest")[0, 0]
        e = self.crop_edge
        if e > 0:
            color = color[e:-e, e:-e]
            depth = depth[e:-e, e:-e]
        pose = self.poses[index]
        pose[:3, 3] *= self.scale  # in place, as datasets.py:112
        return index, color.to(self.color_dtype).contiguous(), depth.contiguous(), pose.to(self.device)

    def prefetch(self, indices=None, workers=4, ahead=8):
        """Frames `indices` (default: all, in order) as dataset[i] returns them, read ahead: `workers`
        processes (torch DataLoader, fork; they run _load_host only, no GPU call) decode up to
        `ahead` frames ahead into pinned host memory, and each frame's H2D copy + normalisation is
        enqueued on a side stream as soon as it arrives, one frame before it is handed out — the
        current stream waits for that frame's work only.  Same values as dataset[i] (same code)."""
        idx = list(range(len(self))) if indices is None else [int(i) for i in indices]
        if not idx:
            return
        dev = torch.device(self.device)
        use_stream = dev.type == "cuda"
        loader = torch.utils.data.DataLoader(
            _HostFrames(self), batch_size=None, sampler=idx, num_workers=workers,
            pin_memory=use_stream, prefetch_factor=max(1, -(-ahead // max(workers, 1))) if workers else None)
        side = torch.cuda.Stream(dev) if use_stream else None
        pending = collections.deque()

        def ready():
            item, ev = pending.popleft()
            if ev is not None:
                torch.cuda.current_stream(dev).wait_event(ev)
                for t in item[1:]:
                    t.record_stream(torch.cuda.current_stream(dev))
            return item

        for i, u8, depth in loader:
            if side is not None:
                side.wait_stream(torch.cuda.current_stream(dev))  # (the LUT, the poses' earlier users)
                with torch.cuda.stream(side):
                    item = self._finish(int(i), u8, depth, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(side)
            else:
                item, ev = self._finish(int(i), u8, depth), None
            pending.append((item, ev))
            if len(pending) > 1:
                yield ready()
        while pending:
            yield ready()


class _HostFrames(torch.utils.data.Dataset):
    """The host half of a BaseDataset (file decode, BaseDataset._load_host) for prefetch workers."""

    def __init__(self, ds):
        self.ds = ds

    def __len__(self):
        return len(self.ds)

    def __getitem__(self, index):
        return (index,) + self.ds._load_host(index)


class Replica(BaseDataset):
    """datasets.py:116-137: results/frame*.jpg, results/depth*.png, traj.txt (one 4×4 per line)."""

    def __init__(self, cfg, args, scale, device="cuda:0", **kw):
        super().__init__(cfg, args, scale, device, **kw)
        self.color_paths = sorted(glob.glob(f"{self.input_folder}/results/frame*.jpg"))
        self.depth_paths = sorted(glob.glob(f"{self.input_folder}/results/depth*.png"))
        self.n_img = len(self.color_paths)
        self.load_poses(f"{self.input_folder}/traj.txt")

    def load_poses(self, path):
        with open(path) as f:
            lines = f.readlines()
        self.poses = [_flip_yz(list(map(float, lines[i].split()))) for i in range(self.n_img)]


class Azure(BaseDataset):
    """datasets.py:140-178 (the Apartment config): color/*.jpg, depth/*.png, scene/trajectory.log
    (5 lines per pose: a header, then the 4×4); identity poses when the log is absent."""

    def __init__(self, cfg, args, scale, device="cuda:0", **kw):
        super().__init__(cfg, args, scale, device, **kw)
        self.color_paths = sorted(glob.glob(os.path.join(self.input_folder, "color", "*.jpg")))
        self.depth_paths = sorted(glob.glob(os.path.join(self.input_folder, "depth", "*.png")))
        self.n_img = len(self.color_paths)
        self.load_poses(os.path.join(self.input_folder, "scene", "trajectory.log"))

    def load_poses(self, path):
        self.poses = []
        if os.path.exists(path):
            with open(path) as f:
                content = f.readlines()
            for i in range(0, len(content), 5):
                self.poses.append(_flip_yz(list(map(float, "".join(content[i + 1:i + 5]).strip().split()))))
        else:
            self.poses = [torch.eye(4) for _ in range(self.n_img)]


class ScanNet(BaseDataset):
    """datasets.py:181-208: frames/color/<n>.jpg, frames/depth/<n>.png, frames/pose/<n>.txt, all
    sorted by the integer file stem."""

    def __init__(self, cfg, args, scale, device="cuda:0", **kw):
        super().__init__(cfg, args, scale, device, **kw)
        self.input_folder = os.path.join(self.input_folder, "frames")
        stem = lambda x: int(os.path.basename(x)[:-4])  # noqa: E731
        self.color_paths = sorted(glob.glob(os.path.join(self.input_folder, "color", "*.jpg")), key=stem)
        self.depth_paths = sorted(glob.glob(os.path.join(self.input_folder, "depth", "*.png")), key=stem)
        self.load_poses(os.path.join(self.input_folder, "pose"))
        self.n_img = len(self.color_paths)

    def load_poses(self, path):
        stem = lambda x: int(os.path.basename(x)[:-4])  # noqa: E731
        self.poses = []
        for p in sorted(glob.glob(os.path.join(path, "*.txt")), key=stem):
            with open(p) as f:
                rows = [list(map(float, line.split(" "))) for line in f.readlines()]
            self.poses.append(_flip_yz(rows))


dataset_dict = {"replica": Replica, "scannet": ScanNet, "azure": Azure}


def get_dataset(cfg, args, scale, device="cuda:0", **kw):
    """datasets.py:47-48."""
    if cfg["dataset"] not in dataset_dict:
        raise NotImplementedError(f"dataset {cfg['dataset']!r} is out of scope (have {sorted(dataset_dict)})")
    return dataset_dict[cfg["dataset"]](cfg, args, scale, device=device, **kw)


# ------------------------------------------------------------------------------------------------
# checkpoints (src/utils/Logger.py:21-35; loaded by NICE_SLAM / Mesher as ckpt['c'], ...)
# ------------------------------------------------------------------------------------------------
def save_checkpoint(path, shared_c, decoders, gt_c2w_list, estimate_c2w_list, keyframe_list, idx,
                    selected_keyframes=None):
    """The reference's ckpt dict, same keys and legacy (non-zip) serialisation (Logger.py:23-32).
    Grids are written as the [1, C, Z, Y, X] tensors they are (channels-last strides survive)."""
    torch.save({"c": shared_c, "decoder_state_dict": decoders.state_dict(), "gt_c2w_list": gt_c2w_list,
                "estimate_c2w_list": estimate_c2w_list, "keyframe_list": keyframe_list,
                "selected_keyframes": selected_keyframes, "idx": idx}, path, _use_new_zipfile_serialization=False)


def load_checkpoint(path, device="cuda:0"):
    """Inverse of save_checkpoint (tensors only: weights_only=True); grids come back channels-last
    on `device`, the layout the HIP kernels read."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    ck["c"] = {k: v.to(device).contiguous(memory_format=torch.channels_last_3d) for k, v in ck["c"].items()}
    return ck
