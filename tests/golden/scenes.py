"""Deterministic synthetic frames shared by the loop-level fixture generator
(tests/golden/make_golden_loop.py, build container) and the tests that replay it (GPU box).

Everything here is plain numpy float64 / integer arithmetic (IEEE-exact, platform independent)
and numpy's PCG64 generator, so both sides rebuild bit-identical images from a seed instead of
storing megabytes of pixels.  Depth is quantised like a sensor PNG (uint16 millimetres / 1000).
"""
from __future__ import annotations

import numpy as np

ROOM0_BOUND = [[-2.9, 8.9], [-3.2, 5.5], [-3.5, 3.3]]       # configs/Replica/room0.yaml:3
ROOM0_CAM = dict(H=680, W=1200, fx=600.0, fy=600.0, cx=599.5, cy=339.5)  # configs/Replica/replica.yaml
TINY_BOUND = [[0.0, 3.0], [-0.5, 2.2], [0.2, 2.5]]           # tests/golden/make_golden.py (tiny_scene.npz)
TINY_CAM = dict(H=96, W=128, fx=60.0, fy=60.0, cx=63.5, cy=47.5)


def look_pose(center, yaw, pitch, offset=(0.0, 0.0, 0.0)):
    """c2w [4,4] float32: camera at center+offset, rotated by yaw (about z) then pitch (about x);
    the camera looks down its -z axis (NICE-SLAM / OpenGL convention, common.py:82)."""
    cy, sy, cp, sp = np.cos(yaw), np.sin(yaw), np.cos(pitch), np.sin(pitch)
    rz = np.array([[cy, -sy, 0.0], [sy, cy, 0.0], [0.0, 0.0, 1.0]])
    rx = np.array([[1.0, 0.0, 0.0], [0.0, cp, -sp], [0.0, sp, cp]])
    m = np.eye(4)
    m[:3, :3] = rz @ rx
    m[:3, 3] = np.asarray(center, dtype=np.float64) + np.asarray(offset, dtype=np.float64)
    return m.astype(np.float32)


def box_depth(c2w, cam, bound, shrink=0.1, seed=0, hole_frac=0.04):
    """Sensor-like depth [H,W] float32: distance along the pixel ray (z-depth, as the sensor
    reports) to the walls of the bound shrunk by `shrink` of its extent, jittered by U(0.9,1.0)
    per pixel, quantised to millimetres, with `hole_frac` zero pixels (gt==0 paths)."""
    H, W = cam["H"], cam["W"]
    fx, fy, cx, cy = cam["fx"], cam["fy"], cam["cx"], cam["cy"]
    b = np.asarray(bound, dtype=np.float64)
    ext = b[:, 1] - b[:, 0]
    lo, hi = b[:, 0] + shrink * ext, b[:, 1] - shrink * ext
    jj, ii = np.meshgrid(np.arange(H, dtype=np.float64), np.arange(W, dtype=np.float64), indexing="ij")
    dirs = np.stack([(ii - cx) / fx, -(jj - cy) / fy, -np.ones_like(ii)], -1)   # z-depth 1 per unit
    R = c2w[:3, :3].astype(np.float64)
    o = c2w[:3, 3].astype(np.float64)
    d = dirs @ R.T
    with np.errstate(divide="ignore", invalid="ignore"):
        t = (np.stack([lo, hi], -1)[None, None] - o[None, None, :, None]) / d[..., None]
    t_exit = np.min(np.max(t, -1), -1)
    rng = np.random.default_rng(seed)
    t_exit = t_exit * (0.9 + 0.1 * rng.random((H, W)))
    t_exit[rng.random((H, W)) < hole_frac] = 0.0
    mm = np.clip(np.round(t_exit * 1000.0), 0, 65535).astype(np.uint16)
    return (mm.astype(np.float32) / np.float32(1000.0))


def color_image(cam, seed):
    """gt colour [H,W,3] float32 in [0,1] (8-bit levels, like a decoded JPEG / 255)."""
    rng = np.random.default_rng(seed)
    u8 = rng.integers(0, 256, size=(cam["H"], cam["W"], 3), dtype=np.uint8)
    return u8.astype(np.float32) / np.float32(255.0)


def enlarge_bound(bound_cfg, div):
    """NICE_SLAM.py:145-150 in numpy (same arithmetic as oracle.enlarge_bound)."""
    b = np.asarray(bound_cfg, dtype=np.float64)
    cells = ((b[:, 1] - b[:, 0]) / div).astype(np.int32) + 1
    b = b.copy()
    b[:, 1] = (cells.astype(np.float32) * np.float32(div)).astype(np.float64) + b[:, 0]
    return b


def room0_window():
    """Room0-shaped keyframe window: 5 keyframe poses + the current pose around the room centre,
    each with its depth / colour seeds."""
    b = enlarge_bound(ROOM0_BOUND, 0.32)
    ctr = b.mean(1)
    poses = [look_pose(ctr, 0.35 * k, 0.15 * ((k % 3) - 1), (0.2 * (k - 2), 0.1 * (k % 2), 0.05 * k))
             for k in range(5)]
    cur = look_pose(ctr, 0.4, 0.05, (0.1, -0.1, 0.0))
    return b, poses, cur


def tiny_window(n_kf=5):
    """Tiny-scene window for the optimize_map fixture: n_kf keyframe poses + the current one."""
    b = enlarge_bound(TINY_BOUND, 0.32)
    ctr = b.mean(1)
    poses = [look_pose(ctr, 0.5 + 0.12 * k, 0.3 + 0.05 * ((k % 3) - 1), (0.05 * (k - 2), -0.03 * k, 0.02 * (k % 2)))
             for k in range(n_kf)]
    cur = look_pose(ctr, 0.5 + 0.12 * n_kf, 0.32, (0.06, -0.04, 0.0))
    return b, poses, cur
