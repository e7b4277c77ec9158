"""Renderer with the reference's call surface (src/utils/Renderer.py), on the HIP kernels.

render_batch_ray = sampler kernel (float64 z) → pts = o + d·z (torch, float64, differentiable in
the rays) → fused query kernel (grid lookups + decoders + OOB logit) → compositing kernel.
"""
from __future__ import annotations

import torch

from . import ops
from .common import get_rays


class Renderer(object):
    def __init__(self, cfg, args, slam, points_batch_size=500000, ray_batch_size=100000):
        self.ray_batch_size = ray_batch_size
        self.points_batch_size = points_batch_size
        r = cfg["rendering"]
        self.lindisp = r["lindisp"]
        self.perturb = r["perturb"]
        self.N_samples = r["N_samples"]
        self.N_surface = r["N_surface"]
        self.N_importance = r["N_importance"]
        self.scale = cfg.get("scale", 1)
        self.occupancy = cfg["occupancy"]
        self.nice = slam.nice
        self.bound = slam.bound
        self.H, self.W, self.fx, self.fy, self.cx, self.cy = slam.H, slam.W, slam.fx, slam.fy, slam.cx, slam.cy
        if not self.nice or not self.occupancy:
            raise NotImplementedError("the HIP path implements NICE-SLAM (nice=True, occupancy=True); iMAP* is "
                                      "out of scope")
        if self.perturb > 0 or self.N_importance > 0:
            raise NotImplementedError("NICE-SLAM renders with perturb=0, N_importance=0 (configs/nice_slam.yaml)")

    def eval_points(self, p, decoders, c=None, stage="color", device="cuda:0"):
        """Renderer.eval_points (Renderer.py:23-61): raw [M,4]; OOB points get occupancy logit 100."""
        return decoders(p, c_grid=c, stage=stage, oob_bound=self.bound)

    def render_batch_ray(self, c, decoders, rays_d, rays_o, device, stage, gt_depth=None, gt_max=None):
        """Renderer.render_batch_ray (Renderer.py:63-198) → (depth f64 [N], uncertainty f64 [N], color f32 [N,3]).

        gt_max (extension): device scalar max(gt_depth) of the full batch when rays are sharded.
        """
        if stage == "coarse":
            gt_depth = None
        n_rays = rays_o.shape[0]
        z = ops.sample_z(rays_o, rays_d, gt_depth, self.bound, self.N_samples, self.N_surface, self.lindisp,
                         gt_max=gt_max)
        pts = rays_o[..., None, :] + rays_d[..., None, :] * z[..., :, None]
        raw = self.eval_points(pts.reshape(-1, 3), decoders, c, stage, device)
        raw = raw.reshape(n_rays, z.shape[1], 4)
        depth, uncertainty, color = ops.composite(raw, z)
        return depth, uncertainty, color

    def render_img(self, c, decoders, c2w, device, stage, gt_depth=None):
        """Renderer.render_img (Renderer.py:200-255): forward-only full-image render in ray batches."""
        with torch.no_grad():
            rays_o, rays_d = get_rays(self.H, self.W, self.fx, self.fy, self.cx, self.cy, c2w, device)
            rays_o = rays_o.reshape(-1, 3)
            rays_d = rays_d.reshape(-1, 3)
            gt = gt_depth.reshape(-1) if gt_depth is not None else None
            ds, us, cs = [], [], []
            for i in range(0, rays_d.shape[0], self.ray_batch_size):
                g = gt[i:i + self.ray_batch_size] if gt is not None else None
                d, u, col = self.render_batch_ray(c, decoders, rays_d[i:i + self.ray_batch_size],
                                                  rays_o[i:i + self.ray_batch_size], device, stage, gt_depth=g)
                ds.append(d.double())
                us.append(u.double())
                cs.append(col)
            return (torch.cat(ds).reshape(self.H, self.W), torch.cat(us).reshape(self.H, self.W),
                    torch.cat(cs).reshape(self.H, self.W, 3))
