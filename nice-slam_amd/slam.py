"""NICE_SLAM set-up pieces that define the hot path's tensors (src/NICE_SLAM.py).

Only what the path needs: camera intrinsics after resize/crop (update_cam, :113-135), the enlarged
float64 bound (load_bound, :137-157), the hierarchical grids (grid_init, :192-250) created
channels-last on the device, and a light state object carrying what Renderer / Tracker / Mapper
read from `slam`.  Process orchestration (:252-307) is out of scope.
"""
from __future__ import annotations

import numpy as np
import torch

from .decoder import NICE


def update_cam(cfg):
    """src/NICE_SLAM.py:113-135 → (H, W, fx, fy, cx, cy)."""
    c = cfg["cam"]
    H, W, fx, fy, cx, cy = c["H"], c["W"], c["fx"], c["fy"], c["cx"], c["cy"]
    if "crop_size" in c:
        sx = c["crop_size"][1] / W
        sy = c["crop_size"][0] / H
        fx, fy, cx, cy = sx * fx, sy * fy, sx * cx, sy * cy
        W, H = c["crop_size"][1], c["crop_size"][0]
    if c["crop_edge"] > 0:
        H -= c["crop_edge"] * 2
        W -= c["crop_edge"] * 2
        cx -= c["crop_edge"]
        cy -= c["crop_edge"]
    return H, W, fx, fy, cx, cy


def load_bound(cfg, scale=None):
    """src/NICE_SLAM.py:145-150: float64 [3,2]; upper end = lo + (int(ext/div)+1)*div (float32 product)."""
    scale = cfg.get("scale", 1) if scale is None else scale
    b = torch.from_numpy(np.array(cfg["mapping"]["bound"], dtype=np.float64) * scale)
    div = cfg["grid_len"]["bound_divisible"]
    cells = ((b[:, 1] - b[:, 0]) / div).int() + 1
    b[:, 1] = (cells.to(torch.float32) * np.float32(div)).to(torch.float64) + b[:, 0]
    return b


def grid_shapes(cfg, bound, coarse=None):
    """[1, C, Z, Y, X] per level (src/NICE_SLAM.py:211-248; extents truncated by int())."""
    coarse = cfg["coarse"] if coarse is None else coarse
    c_dim = cfg["model"]["c_dim"]
    ext = bound[:, 1] - bound[:, 0]
    out = {}
    for k in (["coarse"] if coarse else []) + ["middle", "fine", "color"]:
        enl = cfg["model"]["coarse_bound_enlarge"] if k == "coarse" else 1
        xyz = [int(v) for v in (ext * enl / cfg["grid_len"][k]).tolist()]
        out["grid_" + k] = [1, c_dim, xyz[2], xyz[1], xyz[0]]
    return out


def grid_init(cfg, bound, device="cuda:0", coarse=None, generator=None):
    """Grids ~ N(0, 0.01) (fine N(0, 1e-4)), channels-last on the device (src/NICE_SLAM.py:192-250)."""
    std = {"grid_coarse": 0.01, "grid_middle": 0.01, "grid_fine": 1e-4, "grid_color": 0.01}
    out = {}
    for k, shp in grid_shapes(cfg, bound, coarse).items():
        t = torch.zeros(shp).normal_(0, std[k], generator=generator)
        out[k] = t.to(device).contiguous(memory_format=torch.channels_last_3d)
    return out


def build_decoders(cfg, bound, device="cuda:0"):
    """config.get_model + load_bound's decoder wiring (src/conv_onet/config.py:4-33, NICE_SLAM.py:151-157)."""
    gl = cfg["grid_len"]
    dec = NICE(dim=cfg["data"]["dim"], c_dim=cfg["model"]["c_dim"], coarse=cfg["coarse"],
               coarse_grid_len=gl["coarse"], middle_grid_len=gl["middle"], fine_grid_len=gl["fine"],
               color_grid_len=gl["color"], pos_embedding_method=cfg["model"]["pos_embedding_method"])
    dec.set_bound(bound, cfg["model"]["coarse_bound_enlarge"])
    return dec.to(device)


class SlamState:
    """What Renderer / Tracker / Mapper read from the reference's NICE_SLAM object."""

    def __init__(self, cfg, device="cuda:0", n_img=1, generator=None):
        self.cfg = cfg
        self.nice = True
        self.coarse = cfg["coarse"]
        self.occupancy = cfg["occupancy"]
        self.verbose = cfg.get("verbose", False)
        self.low_gpu_mem = cfg.get("low_gpu_mem", False)
        self.H, self.W, self.fx, self.fy, self.cx, self.cy = update_cam(cfg)
        self.bound = load_bound(cfg)
        self.shared_decoders = build_decoders(cfg, self.bound, device)
        self.shared_c = grid_init(cfg, self.bound, device, generator=generator)
        self.estimate_c2w_list = torch.zeros((n_img, 4, 4))
        self.gt_c2w_list = torch.zeros((n_img, 4, 4))
        self.idx = torch.zeros((1)).int()
        self.mapping_first_frame = torch.zeros((1)).int()
        self.mapping_idx = torch.zeros((1)).int()
        self.mapping_cnt = torch.zeros((1)).int()
        self.output = cfg.get("data", {}).get("output", "output")
        from .renderer import Renderer
        self.renderer = Renderer(cfg, None, self)
