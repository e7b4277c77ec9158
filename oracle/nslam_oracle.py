"""ORACLE — test infrastructure only.

CPU restatement (eager PyTorch, float64/float32 exactly where the reference uses them) of
NICE-SLAM's volumetric-rendering hot path. It is the CHECKER for the HIP path:

  * only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it;
  * the product (``nice-slam_amd/``) never imports or calls it and has no CPU fallback;
  * it is pinned against golden vectors produced by importing the reference's own hot-path modules
    in the build container (``tests/golden/make_golden.py`` → ``tests/golden/*.npz``), see
    ``tests/test_oracle_golden.py``.

Every function cites the reference file:line it restates (paths relative to the reference repo).
Torch is used here purely as a numeric library (autograd gives the VJPs the tests compare). It runs
on CPU as the checker; bench.py's baseline leg also runs it on the device, as the stand-in for the
reference's own PyTorch-on-GPU path (the same torch ops the reference issues).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

STAGES = ("coarse", "middle", "fine", "color")
HIDDEN = 32
EMB = 93


# ----------------------------------------------------------------------------------------------
# scene bound and grid shapes
# ----------------------------------------------------------------------------------------------
def enlarge_bound(bound_cfg, bound_divisible: float, scale: float = 1.0) -> torch.Tensor:
    """src/NICE_SLAM.py:145-150. Returns the float64 [3,2] bound.

    The upper end is lo + (int(ext/div)+1)*div where the product is an int32 tensor times a
    Python float, i.e. it is rounded to float32 before being added to the float64 lower end.
    """
    b = torch.from_numpy(np.asarray(bound_cfg, dtype=np.float64) * scale)
    cells = ((b[:, 1] - b[:, 0]) / bound_divisible).int() + 1
    upper_f32 = cells.to(torch.float32) * np.float32(bound_divisible)
    b[:, 1] = upper_f32.to(torch.float64) + b[:, 0]
    return b


def grid_shape(bound: torch.Tensor, grid_len: float, c_dim: int = 32, enlarge: float = 1.0):
    """src/NICE_SLAM.py:211-248: [1, C, Z, Y, X] with each extent truncated by int()."""
    ext = bound[:, 1] - bound[:, 0]
    xyz = [int(v) for v in (ext * enlarge / grid_len).tolist()]
    return [1, c_dim, xyz[2], xyz[1], xyz[0]]


def make_grids(bound, grid_len: dict, c_dim=32, coarse=True, coarse_enlarge=2.0, gen=None):
    """src/NICE_SLAM.py:192-250 (N(0,0.01) everywhere except fine N(0,1e-4))."""
    std = {"coarse": 0.01, "middle": 0.01, "fine": 1e-4, "color": 0.01}
    out = {}
    for k in (["coarse"] if coarse else []) + ["middle", "fine", "color"]:
        shp = grid_shape(bound, grid_len[k], c_dim, coarse_enlarge if k == "coarse" else 1.0)
        out["grid_" + k] = torch.randn(shp, generator=gen, dtype=torch.float32) * std[k]
    return out


# ----------------------------------------------------------------------------------------------
# decoders (functional form over a state_dict with the reference's key names)
# ----------------------------------------------------------------------------------------------
def normalize_coords(p64: torch.Tensor, bound: torch.Tensor) -> torch.Tensor:
    """src/common.py:269-284 (float64, per axis ((p-lo)/(hi-lo))*2-1)."""
    lo = bound[:, 0]
    ext = bound[:, 1] - bound[:, 0]
    return ((p64 - lo) / ext) * 2 - 1.0


def grid_features(p64, grid, bound):
    """src/conv_onet/models/decoder.py:168-175 → [P, C] (trilinear, border, align_corners)."""
    g = normalize_coords(p64, bound).float().reshape(1, -1, 1, 1, 3)
    f = F.grid_sample(grid, g, mode="bilinear", padding_mode="border", align_corners=True)
    return f.reshape(grid.shape[1], -1).t()


def mlp_xyz(sd, pre, p64, feat):
    """MLP.forward, src/conv_onet/models/decoder.py:177-203 (fourier, 5 blocks, skip after 2)."""
    emb = torch.sin(p64.float() @ sd[pre + "embedder._B"])
    h = emb
    for i in range(5):
        h = F.relu(F.linear(h, sd[f"{pre}pts_linears.{i}.weight"], sd[f"{pre}pts_linears.{i}.bias"]))
        h = h + F.linear(feat, sd[f"{pre}fc_c.{i}.weight"], sd[f"{pre}fc_c.{i}.bias"])
        if i == 2:
            h = torch.cat([emb, h], -1)
    return F.linear(h, sd[pre + "output_linear.weight"], sd[pre + "output_linear.bias"])


def mlp_no_xyz(sd, pre, feat):
    """MLP_no_xyz.forward, src/conv_onet/models/decoder.py:262-274."""
    h = feat
    for i in range(5):
        h = F.relu(F.linear(h, sd[f"{pre}pts_linears.{i}.weight"], sd[f"{pre}pts_linears.{i}.bias"]))
        if i == 2:
            h = torch.cat([feat, h], -1)
    return F.linear(h, sd[pre + "output_linear.weight"], sd[pre + "output_linear.bias"])


def nice_raw(sd, p64, grids, stage, bound, coarse_bound=None):
    """NICE.forward stage combiner, src/conv_onet/models/decoder.py:312-342 → raw [P,4] f32."""
    P = p64.shape[0]
    zeros = torch.zeros(P, 3, dtype=torch.float32, device=p64.device)
    if stage == "coarse":
        cb = coarse_bound if coarse_bound is not None else bound * 2
        occ = mlp_no_xyz(sd, "coarse_decoder.", grid_features(p64, grids["grid_coarse"], cb))[:, 0]
        return torch.cat([zeros, occ[:, None]], 1)
    f_mid = grid_features(p64, grids["grid_middle"], bound)
    occ = mlp_xyz(sd, "middle_decoder.", p64, f_mid)[:, 0]
    if stage == "middle":
        return torch.cat([zeros, occ[:, None]], 1)
    f_fine = torch.cat([grid_features(p64, grids["grid_fine"], bound), f_mid.detach()], 1)
    occ = mlp_xyz(sd, "fine_decoder.", p64, f_fine)[:, 0] + occ
    if stage == "fine":
        return torch.cat([zeros, occ[:, None]], 1)
    rgb = mlp_xyz(sd, "color_decoder.", p64, grid_features(p64, grids["grid_color"], bound))[:, :3]
    return torch.cat([rgb, occ[:, None]], 1)


def eval_points(sd, p64, grids, stage, bound, coarse_bound=None):
    """Renderer.eval_points, src/utils/Renderer.py:23-61: strict-inequality OOB ⇒ occ logit 100."""
    inside = ((p64 > bound[:, 0]) & (p64 < bound[:, 1])).all(1)
    raw = nice_raw(sd, p64, grids, stage, bound, coarse_bound)
    occ = torch.where(inside, raw[:, 3], torch.full_like(raw[:, 3], 100.0))
    return torch.cat([raw[:, :3], occ[:, None]], 1)


# ----------------------------------------------------------------------------------------------
# sampler, compositing, render
# ----------------------------------------------------------------------------------------------
def far_bound(rays_o, rays_d, bound):
    """AABB exit distance, src/utils/Renderer.py:98-105 (also Tracker.py:95-99, Mapper.py:471-476)."""
    o = rays_o.detach().double()[:, :, None]
    d = rays_d.detach().double()[:, :, None]
    t = (bound[None] - o) / d
    return t.max(2).values.min(1).values


def sample_z(rays_o, rays_d, gt_depth, bound, n_strat, n_surf, lindisp=False, gt_max=None):
    """Stratified + surface sampler, src/utils/Renderer.py:82-170 (perturb=0) → z [N,S] f64.

    gt_max: max(gt_depth) of the FULL batch when this call sees only a shard of it."""
    with torch.no_grad():
        far_bb = far_bound(rays_o, rays_d, bound)[:, None] + 0.01
        dev = rays_o.device
        t_s = torch.linspace(0.0, 1.0, n_strat, device=dev)
        if gt_depth is None:
            n_surf = 0
            near = 0.01
            far = far_bb
        else:
            gt = gt_depth.reshape(-1, 1)
            near = gt.repeat(1, n_strat) * 0.01
            gmax = torch.max(gt) if gt_max is None else gt_max.reshape(()).float()
            far = torch.clamp(far_bb, 0, gmax * 1.2)
        if lindisp:
            z = 1.0 / (1.0 / near * (1.0 - t_s) + 1.0 / far * t_s)
        else:
            z = near * (1.0 - t_s) + far * t_s
        if n_surf > 0:
            t_u = torch.linspace(0.0, 1.0, n_surf, device=dev).double()
            pos = (gt > 0)[:, 0]
            zs = torch.zeros(gt.shape[0], n_surf, dtype=torch.float64, device=dev)
            g = gt[pos]
            zs[pos] = (0.95 * g) * (1.0 - t_u) + (1.05 * g) * t_u
            zs[~pos] = 0.001 * (1.0 - t_u) + gmax * t_u
            z = torch.sort(torch.cat([z, zs], -1), -1).values
    return z


def composite(raw, z, occupancy=True):
    """raw2outputs_nerf_color, src/common.py:204-245 (occupancy mode) → depth f64, var f64, rgb f32."""
    assert occupancy, "only occupancy=True is on the NICE-SLAM path (configs/nice_slam.yaml:5)"
    alpha = torch.sigmoid(10 * raw[..., 3])
    ones = torch.ones_like(alpha[:, :1])
    trans = torch.cumprod(torch.cat([ones, 1.0 - alpha + 1e-10], -1), -1)[:, :-1]
    w = alpha * trans
    rgb = torch.sum(w[..., None] * raw[..., :3], -2)
    depth = torch.sum(w * z, -1)
    dz = z - depth[:, None]
    var = torch.sum(w * dz * dz, 1)
    return depth, var, rgb, w


def render_batch_ray(sd, grids, rays_d, rays_o, stage, bound, gt_depth=None,
                     n_strat=32, n_surf=16, coarse_bound=None, return_z=False, gt_max=None):
    """Renderer.render_batch_ray, src/utils/Renderer.py:63-198 (N_importance=0, perturb=0)."""
    if stage == "coarse":
        gt_depth = None
    z = sample_z(rays_o, rays_d, gt_depth, bound, n_strat, n_surf, gt_max=gt_max)
    pts = rays_o[:, None, :] + rays_d[:, None, :] * z[:, :, None]
    raw = eval_points(sd, pts.reshape(-1, 3), grids, stage, bound, coarse_bound)
    depth, var, rgb, _ = composite(raw.reshape(z.shape[0], z.shape[1], 4), z)
    if return_z:
        return depth, var, rgb, z
    return depth, var, rgb


# ----------------------------------------------------------------------------------------------
# rays / camera / losses (host-side pieces of the path)
# ----------------------------------------------------------------------------------------------
def rays_from_uv(i, j, c2w, fx, fy, cx, cy):
    """get_rays_from_uv, src/common.py:74-89."""
    dirs = torch.stack([(i - cx) / fx, -(j - cy) / fy, -torch.ones_like(i)], -1)
    rays_d = torch.sum(dirs[:, None, :] * c2w[:3, :3], -1)
    rays_o = c2w[:3, -1].expand(rays_d.shape)
    return rays_o, rays_d


def quat_to_rot(q):
    """quad2rotation, src/common.py:137-160 (device-agnostic restatement; [B,4] (w,x,y,z))."""
    w, x, y, z = q.unbind(-1)
    s = 2.0 / (q * q).sum(-1)
    rows = [
        1 - s * (y * y + z * z), s * (x * y - z * w), s * (x * z + y * w),
        s * (x * y + z * w), 1 - s * (x * x + z * z), s * (y * z - x * w),
        s * (x * z - y * w), s * (y * z + x * w), 1 - s * (x * x + y * y),
    ]
    return torch.stack(rows, -1).reshape(q.shape[:-1] + (3, 3))


def camera_from_tensor(t):
    """get_camera_from_tensor, src/common.py:163-176 → [3,4]."""
    single = t.dim() == 1
    tt = t[None] if single else t
    rt = torch.cat([quat_to_rot(tt[:, :4]), tt[:, 4:, None]], 2)
    return rt[0] if single else rt


def tracker_loss(depth, var, color, gt_depth, gt_color, handle_dynamic=True, w_color=0.5,
                 use_color=True):
    """Tracker.optimize_cam_in_batch loss, src/Tracker.py:110-123."""
    var = var.detach()
    r = torch.abs(gt_depth - depth) / torch.sqrt(var + 1e-10)
    if handle_dynamic:
        keep = (r < 10 * r.median()) & (gt_depth > 0)
    else:
        keep = gt_depth > 0
    loss = r[keep].sum()
    if use_color:
        loss = loss + w_color * torch.abs(gt_color - color)[keep].sum()
    return loss


def mapper_loss(depth, color, gt_depth, gt_color, stage, w_color=0.2):
    """Mapper.optimize_map loss, src/Mapper.py:487-493."""
    m = gt_depth > 0
    loss = torch.abs(gt_depth[m] - depth[m]).sum()
    if stage == "color":
        loss = loss + w_color * torch.abs(gt_color - color).sum()
    return loss


def inside_mask(rays_o, rays_d, gt_depth, bound):
    """Ray prefilter, src/Tracker.py:93-100 / src/Mapper.py:469-477: t_exit >= gt_depth."""
    return far_bound(rays_o, rays_d, bound) >= gt_depth


# ----------------------------------------------------------------------------------------------
# decoder state_dict construction (reference init, src/conv_onet/models/decoder.py:70-79,149-159)
# ----------------------------------------------------------------------------------------------
def init_decoders(gen=None, coarse=True, c_dim=32):
    """Seeded params with the reference's key names and init laws (xavier-uniform, zero bias for
    DenseLayer; nn.Linear default for fc_c; B ~ N(0,1)*25)."""
    sd = {}

    def dense(name, fan_in, fan_out, gain):
        a = gain * math.sqrt(6.0 / (fan_in + fan_out))
        sd[name + ".weight"] = (torch.rand(fan_out, fan_in, generator=gen) * 2 - 1) * a
        sd[name + ".bias"] = torch.zeros(fan_out)

    def linear(name, fan_in, fan_out):
        k = 1.0 / math.sqrt(fan_in)
        sd[name + ".weight"] = (torch.rand(fan_out, fan_in, generator=gen) * 2 - 1) * k
        sd[name + ".bias"] = (torch.rand(fan_out, generator=gen) * 2 - 1) * k

    relu_gain = math.sqrt(2.0)
    if coarse:
        for i, fin in enumerate([32, 32, 32, 32 + c_dim, 32]):
            dense(f"coarse_decoder.pts_linears.{i}", fin, 32, relu_gain)
        dense("coarse_decoder.output_linear", 32, 1, 1.0)
    for dec, cin, nout in (("middle", c_dim, 1), ("fine", 2 * c_dim, 1), ("color", c_dim, 4)):
        pre = f"{dec}_decoder."
        for i in range(5):
            linear(f"{pre}fc_c.{i}", cin, 32)
        sd[pre + "embedder._B"] = torch.randn(3, EMB, generator=gen) * 25
        for i, fin in enumerate([EMB, 32, 32, 32 + EMB, 32]):
            dense(f"{pre}pts_linears.{i}", fin, 32, relu_gain)
        dense(pre + "output_linear", 32, nout, 1.0)
    return sd
