"""Host-side pieces of the path with the reference's names (src/common.py).

Ray generation, pixel selection and the pose parametrisation are tiny [N,3]/[7]-sized tensor
programs: they stay torch ops on the device (graph-capturable, differentiable w.r.t. the camera
tensor).  Compositing is the HIP kernel (ops.composite).
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops


def as_intrinsics_matrix(intrinsics):
    """src/common.py:6-16."""
    K = np.eye(3)
    K[0, 0], K[1, 1], K[0, 2], K[1, 2] = intrinsics[0], intrinsics[1], intrinsics[2], intrinsics[3]
    return K


def random_select(l, k):
    """src/common.py:66-71: k random indices of range(l) (numpy RNG, as the reference)."""
    return list(np.random.permutation(np.array(range(l)))[:min(l, k)])


def get_rays_from_uv(i, j, c2w, H, W, fx, fy, cx, cy, device):
    """src/common.py:74-89: dirs=((i-cx)/fx, -(j-cy)/fy, -1); rays_d = R dirs; rays_o = t."""
    if isinstance(c2w, np.ndarray):
        c2w = torch.from_numpy(c2w)
    c2w = c2w.to(device)
    dirs = torch.stack([(i - cx) / fx, -(j - cy) / fy, -torch.ones_like(i)], -1).to(device)
    rays_d = torch.sum(dirs[:, None, :] * c2w[:3, :3], -1)
    rays_o = c2w[:3, -1].expand(rays_d.shape)
    return rays_o, rays_d


def select_uv(i, j, n, depth, color, device="cuda:0", generator=None):
    """src/common.py:92-107 (uniform random pixels via torch.randint on the device)."""
    i = i.reshape(-1)
    j = j.reshape(-1)
    idx = torch.randint(i.shape[0], (n,), device=device, generator=generator)
    return i[idx], j[idx], depth.reshape(-1)[idx], color.reshape(-1, 3)[idx]


def get_sample_uv(H0, H1, W0, W1, n, depth, color, device="cuda:0", generator=None):
    """src/common.py:110-122."""
    depth = depth[H0:H1, W0:W1]
    color = color[H0:H1, W0:W1]
    i, j = torch.meshgrid(torch.linspace(W0, W1 - 1, W1 - W0, device=device),
                          torch.linspace(H0, H1 - 1, H1 - H0, device=device), indexing="ij")
    return select_uv(i.t(), j.t(), n, depth, color, device=device, generator=generator)


def get_samples(H0, H1, W0, W1, n, H, W, fx, fy, cx, cy, c2w, depth, color, device, generator=None):
    """src/common.py:125-134."""
    i, j, d, c = get_sample_uv(H0, H1, W0, W1, n, depth, color, device=device, generator=generator)
    rays_o, rays_d = get_rays_from_uv(i, j, c2w, H, W, fx, fy, cx, cy, device)
    return rays_o, rays_d, d, c


def get_rays(H, W, fx, fy, cx, cy, c2w, device):
    """src/common.py:248-266 (rays of a whole image)."""
    if isinstance(c2w, np.ndarray):
        c2w = torch.from_numpy(c2w)
    c2w = c2w.to(device)
    i, j = torch.meshgrid(torch.linspace(0, W - 1, W, device=device), torch.linspace(0, H - 1, H, device=device),
                          indexing="ij")
    i, j = i.t(), j.t()
    dirs = torch.stack([(i - cx) / fx, -(j - cy) / fy, -torch.ones_like(i)], -1)
    rays_d = torch.sum(dirs[..., None, :] * c2w[:3, :3], -1)
    rays_o = c2w[:3, -1].expand(rays_d.shape)
    return rays_o, rays_d


def quad2rotation(quad):
    """src/common.py:137-160 — quaternion (w,x,y,z), unnormalised (2/|q|^2), device-agnostic."""
    qr, qi, qj, qk = quad[:, 0], quad[:, 1], quad[:, 2], quad[:, 3]
    two_s = 2.0 / (quad * quad).sum(-1)
    rows = [1 - two_s * (qj ** 2 + qk ** 2), two_s * (qi * qj - qk * qr), two_s * (qi * qk + qj * qr),
            two_s * (qi * qj + qk * qr), 1 - two_s * (qi ** 2 + qk ** 2), two_s * (qj * qk - qi * qr),
            two_s * (qi * qk - qj * qr), two_s * (qj * qk + qi * qr), 1 - two_s * (qi ** 2 + qj ** 2)]
    return torch.stack(rows, -1).reshape(-1, 3, 3)


def get_camera_from_tensor(inputs):
    """src/common.py:163-176: [7] (or [B,7]) quaternion+translation → [3,4] (or [B,3,4])."""
    single = inputs.dim() == 1
    x = inputs[None] if single else inputs
    RT = torch.cat([quad2rotation(x[:, :4]), x[:, 4:, None]], 2)
    return RT[0] if single else RT


def get_tensor_from_camera(RT, Tquad=False):
    """src/common.py:179-201 without mathutils: rotation → quaternion (w,x,y,z), w >= 0.

    The reference calls Blender's mathutils Matrix.to_quaternion() (not installed here); q and -q
    are the same rotation and Adam on the 7-vector is odd-symmetric, so the sign convention does
    not change the optimised pose.  Parity with mathutils itself is unpinned (absent library).
    """
    dev = RT.device if torch.is_tensor(RT) else None
    M = RT.detach().cpu().double().numpy() if torch.is_tensor(RT) else np.asarray(RT, dtype=np.float64)
    R, T = M[:3, :3], M[:3, 3]
    tr = R[0, 0] + R[1, 1] + R[2, 2]
    if tr > 0:
        s = 2.0 * np.sqrt(tr + 1.0)
        q = [0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s]
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = 2.0 * np.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2])
        q = [(R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s]
    elif R[1, 1] > R[2, 2]:
        s = 2.0 * np.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2])
        q = [(R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s]
    else:
        s = 2.0 * np.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1])
        q = [(R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s]
    q = np.asarray(q)
    q = q / np.linalg.norm(q)
    if q[0] < 0:
        q = -q
    vec = np.concatenate([T, q]) if Tquad else np.concatenate([q, T])
    out = torch.from_numpy(vec).float()
    return out.to(dev) if dev is not None else out


def camera_tensors(RT):
    """get_tensor_from_camera for a batch of poses [B, 3|4, 4] on their device, without a host round trip:
    the same branch rule and float64 arithmetic as get_tensor_from_camera (rotation → quaternion
    (w,x,y,z) normalised, w >= 0, then T), as float32 [B, 7]."""
    M = RT.detach().to(torch.float64)
    R, T = M[:, :3, :3], M[:, :3, 3]
    r00, r01, r02 = R[:, 0, 0], R[:, 0, 1], R[:, 0, 2]
    r10, r11, r12 = R[:, 1, 0], R[:, 1, 1], R[:, 1, 2]
    r20, r21, r22 = R[:, 2, 0], R[:, 2, 1], R[:, 2, 2]
    tr = r00 + r11 + r22
    cands = []
    s = 2.0 * torch.sqrt((tr + 1.0).clamp_min(0))
    cands.append(torch.stack([0.25 * s, (r21 - r12) / s, (r02 - r20) / s, (r10 - r01) / s], -1))
    s = 2.0 * torch.sqrt((1.0 + r00 - r11 - r22).clamp_min(0))
    cands.append(torch.stack([(r21 - r12) / s, 0.25 * s, (r01 + r10) / s, (r02 + r20) / s], -1))
    s = 2.0 * torch.sqrt((1.0 + r11 - r00 - r22).clamp_min(0))
    cands.append(torch.stack([(r02 - r20) / s, (r01 + r10) / s, 0.25 * s, (r12 + r21) / s], -1))
    s = 2.0 * torch.sqrt((1.0 + r22 - r00 - r11).clamp_min(0))
    cands.append(torch.stack([(r10 - r01) / s, (r02 + r20) / s, (r12 + r21) / s, 0.25 * s], -1))
    c0 = (tr > 0)[:, None]
    c1 = ((r00 > r11) & (r00 > r22))[:, None]
    c2 = (r11 > r22)[:, None]
    q = torch.where(c0, cands[0], torch.where(c1, cands[1], torch.where(c2, cands[2], cands[3])))
    q = q / torch.sqrt((q * q).sum(-1, keepdim=True))
    q = torch.where(q[:, :1] < 0, -q, q)
    return torch.cat([q, T], -1).float()


def raw2outputs_nerf_color(raw, z_vals, rays_d, occupancy=False, device="cuda:0"):
    """src/common.py:204-245 → (depth, var, rgb, weights); occupancy mode on the HIP kernel.

    `weights` is recomputed by the kernel's backward and not materialised; it is returned as None
    (no caller on the NICE-SLAM path uses it: N_importance = 0).
    """
    if not occupancy:
        raise NotImplementedError("NICE-SLAM composites in occupancy mode (configs/nice_slam.yaml:5)")
    depth, var, rgb = ops.composite(raw, z_vals)
    return depth, var, rgb, None


def normalize_3d_coordinate(p, bound):
    """src/common.py:269-284 (float64 arithmetic, out of place)."""
    p = p.reshape(-1, 3)
    lo = bound[:, 0].to(p.device, p.dtype)
    ext = (bound[:, 1] - bound[:, 0]).to(p.device, p.dtype)
    return ((p - lo) / ext) * 2 - 1.0
