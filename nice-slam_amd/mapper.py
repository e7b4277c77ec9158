"""Mapper drop-in: map optimisation on the HIP render path (src/Mapper.py).

`optimize_map` keeps the reference's signature and semantics (Mapper.py:230-540): staged
middle → fine → colour schedule, Adam re-created per call, frustum-masked grid parameters,
optional bundle adjustment of keyframe cameras.  Differences (none changes the maths):
  * keyframe images stay resident on the device (the reference copies them host→device every
    iteration, Mapper.py:439-440);
  * the frustum voxel mask (Mapper.py:93-164) is computed with torch on the device; cv2.remap's
    bilinear lookup is emulated including its 1/32-pixel fixed-point positions and zero border
    (OpenCV is not installed: parity with cv2 itself is unpinned);
  * decoder parameters that are not optimised get requires_grad=False for the call, so the
    fused backward skips their (never used) weight gradients.
The mapping loop driver (Mapper.run, Mapper.py:542-657) is out of scope (dataset/meshing/ckpt glue).
"""
from __future__ import annotations

import numpy as np
import torch

from .common import get_camera_from_tensor, get_samples, get_tensor_from_camera, random_select


def _remap_bilinear(img, u, v):
    """cv2.remap(img, u, v, INTER_LINEAR, BORDER_CONSTANT=0) for float32 maps (INTER_BITS=5)."""
    H, W = img.shape
    X = torch.round(u.clamp(-1e8, 1e8) * 32).to(torch.int64)
    Y = torch.round(v.clamp(-1e8, 1e8) * 32).to(torch.int64)
    x0, y0 = torch.div(X, 32, rounding_mode="floor"), torch.div(Y, 32, rounding_mode="floor")
    fx = (X - x0 * 32).to(torch.float32) / 32
    fy = (Y - y0 * 32).to(torch.float32) / 32

    def tap(x, y):
        ok = (x >= 0) & (x < W) & (y >= 0) & (y < H)
        return torch.where(ok, img[y.clamp(0, H - 1), x.clamp(0, W - 1)], torch.zeros((), device=img.device))

    w00, w01 = (1 - fx) * (1 - fy), fx * (1 - fy)
    w10, w11 = (1 - fx) * fy, fx * fy
    return tap(x0, y0) * w00 + tap(x0 + 1, y0) * w01 + tap(x0, y0 + 1) * w10 + tap(x0 + 1, y0 + 1) * w11


def frustum_mask(c2w, key, val_shape, depth, bound, H, W, fx, fy, cx, cy):
    """Mapper.get_mask_from_c2w (Mapper.py:93-164) on the device: bool mask [X, Y, Z] of the
    grid voxels inside the camera frustum up to the observed depth + 0.5 m, or within 0.5 m of
    the camera.  val_shape = (Z, Y, X)."""
    dev = depth.device
    nz, ny, nx = val_shape[0], val_shape[1], val_shape[2]
    if key == "grid_coarse":
        return torch.ones(nx, ny, nz, dtype=torch.bool, device=dev)
    b = bound
    X, Y, Z = torch.meshgrid(torch.linspace(float(b[0][0]), float(b[0][1]), nx, device=dev),
                             torch.linspace(float(b[1][0]), float(b[1][1]), ny, device=dev),
                             torch.linspace(float(b[2][0]), float(b[2][1]), nz, device=dev), indexing="ij")
    points = torch.stack([X, Y, Z], dim=-1).reshape(-1, 3)
    c2w = c2w.to(dev).float()
    if c2w.shape[0] == 3:
        c2w = torch.cat([c2w, torch.tensor([[0, 0, 0, 1.0]], device=dev)], 0)
    w2c = torch.linalg.inv(c2w)
    cam = points @ w2c[:3, :3].T + w2c[:3, 3]
    cam = cam.double()
    cam[:, 0] *= -1
    K = torch.tensor([[fx, 0.0, cx], [0.0, fy, cy], [0.0, 0.0, 1.0]], dtype=torch.float64, device=dev)
    uvz = cam @ K.T
    z = uvz[:, 2] + 1e-5
    uv = (uvz[:, :2] / z[:, None]).float()
    depths = _remap_bilinear(depth.float(), uv[:, 0], uv[:, 1])
    mask = (uv[:, 0] < W) & (uv[:, 0] > 0) & (uv[:, 1] < H) & (uv[:, 1] > 0)
    depths = torch.where(depths == 0, depths.max(), depths)
    mask = mask & (0 <= -z) & (-z <= depths.double() + 0.5)
    ray_o = c2w[:3, 3]
    d = points - ray_o
    mask = mask | ((d * d).sum(1) < 0.5 * 0.5)
    return mask.reshape(nx, ny, nz)


class Mapper(object):
    def __init__(self, cfg, args, slam, coarse_mapper=False, generator=None):
        self.cfg = cfg
        self.args = args
        self.coarse_mapper = coarse_mapper
        self.nice = slam.nice
        self.c = slam.shared_c
        self.bound = slam.bound
        self.renderer = slam.renderer
        self.decoders = slam.shared_decoders
        self.estimate_c2w_list = slam.estimate_c2w_list
        self.coarse = cfg["coarse"]
        self.occupancy = cfg["occupancy"]
        m = cfg["mapping"]
        self.device = m["device"]
        self.fix_fine = m["fix_fine"]
        self.BA = False
        self.BA_cam_lr = m["BA_cam_lr"]
        self.fix_color = m["fix_color"]
        self.mapping_pixels = m["pixels"]
        self.num_joint_iters = m["iters"]
        self.w_color_loss = m["w_color_loss"]
        self.fine_iter_ratio = m["fine_iter_ratio"]
        self.middle_iter_ratio = m["middle_iter_ratio"]
        self.mapping_window_size = m["mapping_window_size"]
        self.frustum_feature_selection = m["frustum_feature_selection"]
        self.keyframe_selection_method = m["keyframe_selection_method"]
        if self.nice and coarse_mapper:
            self.keyframe_selection_method = "global"
        self.keyframe_dict = []
        self.keyframe_list = []
        self.H, self.W, self.fx, self.fy, self.cx, self.cy = slam.H, slam.W, slam.fx, slam.fy, slam.cx, slam.cy
        self.generator = generator
        self.stage = "middle"
        self.loss_history = None  # set to [] to record per-iteration losses (detached, no host sync)

    # ------------------------------------------------------------------------------------------
    def get_mask_from_c2w(self, c2w, key, val_shape, depth):
        """Frustum voxel selection (Mapper.py:93-164) → bool mask [X, Y, Z] on the device."""
        return frustum_mask(c2w, key, val_shape, depth, self.bound, self.H, self.W, self.fx, self.fy, self.cx,
                            self.cy)

    def keyframe_overlap_scores(self, gt_color, gt_depth, c2w, keyframe_dict, N_samples=16, pixels=100):
        """Mapper.py:185-221: per keyframe, the fraction of the current frame's near-surface samples
        (100 pixels × 16 depths in [0.8·d, d + 0.5]) that project inside it (20-px margin, in front
        of the camera).  One host sync for all keyframes (the reference's loop is host numpy)."""
        dev = self.device
        H, W, fx, fy, cx, cy = self.H, self.W, self.fx, self.fy, self.cx, self.cy
        rays_o, rays_d, gd, _ = get_samples(0, H, 0, W, pixels, H, W, fx, fy, cx, cy, c2w, gt_depth, gt_color, dev,
                                            generator=self.generator)
        if not keyframe_dict:
            return []
        gd = gd.reshape(-1, 1).repeat(1, N_samples)
        t = torch.linspace(0.0, 1.0, N_samples, device=dev)
        z = gd * 0.8 * (1.0 - t) + (gd + 0.5) * t
        verts = (rays_o[..., None, :] + rays_d[..., None, :] * z[..., :, None]).reshape(-1, 3)
        K = torch.tensor([[fx, 0.0, cx], [0.0, fy, cy], [0.0, 0.0, 1.0]], dtype=torch.float64, device=dev)
        counts = []
        for kf in keyframe_dict:
            w2c = torch.linalg.inv(kf["est_c2w"].to(dev).float())
            cam = (verts @ w2c[:3, :3].T + w2c[:3, 3]).double()
            cam[:, 0] *= -1
            uvz = cam @ K.T
            zz = uvz[:, 2] + 1e-5
            uv = (uvz[:, :2] / zz[:, None]).float()
            edge = 20
            m = (uv[:, 0] < W - edge) & (uv[:, 0] > edge) & (uv[:, 1] < H - edge) & (uv[:, 1] > edge) & (zz < 0)
            counts.append(m.sum())
        n = verts.shape[0]
        # mask.sum() / uv.shape[0] as the reference divides: an integer count over the sample count
        return [int(cnt) / n for cnt in torch.stack(counts).cpu()]

    def keyframe_selection_overlap(self, gt_color, gt_depth, c2w, keyframe_dict, k, N_samples=16, pixels=100):
        """Mapper.py:166-228: keyframes whose frustum sees the current frame's surface samples,
        ranked by overlap (stable sort, as `sorted`), then a random permutation (numpy RNG) of the
        ones with any overlap, truncated to k."""
        scores = self.keyframe_overlap_scores(gt_color, gt_depth, c2w, keyframe_dict, N_samples, pixels)
        ranked = sorted(enumerate(scores), key=lambda s: s[1], reverse=True)
        sel = [kid for kid, s in ranked if s > 0.0]
        return list(np.random.permutation(np.array(sel))[:k])

    # ------------------------------------------------------------------------------------------
    def _frame_images(self, kf):
        if "_dev" not in kf:  # keyframe images resident on the device (one copy per keyframe)
            kf["_dev"] = (kf["depth"].to(self.device), kf["color"].to(self.device).float())
        return kf["_dev"]

    def optimize_map(self, num_joint_iters, lr_factor, idx, cur_gt_color, cur_gt_depth, gt_cur_c2w, keyframe_dict,
                     keyframe_list, cur_c2w):
        """Mapping iterations (Mapper.py:230-540); returns the BA-updated cur_c2w or None."""
        H, W, fx, fy, cx, cy = self.H, self.W, self.fx, self.fy, self.cx, self.cy
        c, cfg, device = self.c, self.cfg, self.device
        bottom = torch.tensor([[0, 0, 0, 1.0]], dtype=torch.float32, device=device)
        cur_gt_depth = cur_gt_depth.to(device)
        cur_gt_color = cur_gt_color.to(device).float()
        cur_c2w = cur_c2w.to(device)

        if len(keyframe_dict) == 0:
            optimize_frame = []
        elif self.keyframe_selection_method == "global":
            optimize_frame = random_select(len(self.keyframe_dict) - 1, self.mapping_window_size - 2)
        else:
            optimize_frame = self.keyframe_selection_overlap(cur_gt_color, cur_gt_depth, cur_c2w, keyframe_dict[:-1],
                                                             self.mapping_window_size - 2)
        oldest_frame = None
        if len(keyframe_list) > 0:
            optimize_frame = optimize_frame + [len(keyframe_list) - 1]
            oldest_frame = min(optimize_frame)
        optimize_frame += [-1]
        pixs_per_image = self.mapping_pixels // len(optimize_frame)

        groups = {"decoders": [], "coarse": [], "middle": [], "fine": [], "color": []}
        masked = {}
        for key, val in c.items():
            if self.frustum_feature_selection:
                mask = self.get_mask_from_c2w(cur_c2w, key, val.shape[2:], cur_gt_depth)
                mask = mask.permute(2, 1, 0)[None, None].expand(1, val.shape[1], -1, -1, -1)
                vg = val.detach()[mask].clone().requires_grad_(True)
                masked[key] = (vg, mask)
                groups[key[5:]].append(vg)
            else:
                val = val.detach().requires_grad_(True)
                c[key] = val
                groups[key[5:]].append(val)
        trainable = []
        if not self.fix_fine:
            trainable += list(self.decoders.fine_decoder.parameters())
        if not self.fix_color:
            trainable += list(self.decoders.color_decoder.parameters())
        groups["decoders"] = trainable
        saved_rg = {p: p.requires_grad for p in self.decoders.parameters()}
        ids = {id(p) for p in trainable}
        for p in self.decoders.parameters():
            p.requires_grad_(id(p) in ids)

        cam_tensors = []
        if self.BA:
            for frame in optimize_frame:
                if frame != oldest_frame:
                    c2w = keyframe_dict[frame]["est_c2w"] if frame != -1 else cur_c2w
                    cam_tensors.append(get_tensor_from_camera(c2w).to(device).requires_grad_(True))
        pg = [{"params": groups["decoders"], "lr": 0}, {"params": groups["coarse"], "lr": 0},
              {"params": groups["middle"], "lr": 0}, {"params": groups["fine"], "lr": 0},
              {"params": groups["color"], "lr": 0}]
        if self.BA:
            pg.append({"params": cam_tensors, "lr": 0})
        optimizer = torch.optim.Adam(pg)

        bound = self.bound.to(device)
        for joint_iter in range(num_joint_iters):
            if self.frustum_feature_selection:
                for key, val in c.items():
                    if (self.coarse_mapper and "coarse" in key) or (not self.coarse_mapper and "coarse" not in key):
                        vg, mask = masked[key]
                        val = val.detach()
                        val[mask] = vg
                        c[key] = val
            if self.coarse_mapper:
                self.stage = "coarse"
            elif joint_iter <= int(num_joint_iters * self.middle_iter_ratio):
                self.stage = "middle"
            elif joint_iter <= int(num_joint_iters * self.fine_iter_ratio):
                self.stage = "fine"
            else:
                self.stage = "color"
            st = cfg["mapping"]["stage"][self.stage]
            for gi, name in enumerate(("decoders", "coarse", "middle", "fine", "color")):
                optimizer.param_groups[gi]["lr"] = st[name + "_lr"] * lr_factor
            if self.BA and self.stage == "color":
                optimizer.param_groups[5]["lr"] = self.BA_cam_lr

            optimizer.zero_grad()
            ro_l, rd_l, gd_l, gc_l = [], [], [], []
            cam_id = 0
            for frame in optimize_frame:
                if frame != -1:
                    gt_depth, gt_color = self._frame_images(keyframe_dict[frame])
                    if self.BA and frame != oldest_frame:
                        c2w = get_camera_from_tensor(cam_tensors[cam_id])
                        cam_id += 1
                    else:
                        c2w = keyframe_dict[frame]["est_c2w"].to(device)
                else:
                    gt_depth, gt_color = cur_gt_depth, cur_gt_color
                    c2w = get_camera_from_tensor(cam_tensors[cam_id]) if self.BA else cur_c2w.to(device)
                ro, rd, gd, gc = get_samples(0, H, 0, W, pixs_per_image, H, W, fx, fy, cx, cy, c2w, gt_depth,
                                             gt_color, device, generator=self.generator)
                ro_l.append(ro.float())
                rd_l.append(rd.float())
                gd_l.append(gd.float())
                gc_l.append(gc.float())
            rays_o, rays_d = torch.cat(ro_l), torch.cat(rd_l)
            gt_d, gt_c = torch.cat(gd_l), torch.cat(gc_l)
            with torch.no_grad():  # Mapper.py:469-481
                t = (bound.unsqueeze(0) - rays_o.detach().unsqueeze(-1)) / rays_d.detach().unsqueeze(-1)
                keep = torch.min(torch.max(t, dim=2)[0], dim=1)[0] >= gt_d
            rays_o, rays_d, gt_d, gt_c = rays_o[keep], rays_d[keep], gt_d[keep], gt_c[keep]
            depth, uncertainty, color = self.renderer.render_batch_ray(
                c, self.decoders, rays_d, rays_o, device, self.stage, gt_depth=None if self.coarse_mapper else gt_d)
            dm = gt_d > 0
            loss = torch.abs(gt_d[dm] - depth[dm]).sum()
            if self.stage == "color":
                loss = loss + self.w_color_loss * torch.abs(gt_c - color).sum()
            loss.backward(retain_graph=False)
            if self.loss_history is not None:
                self.loss_history.append(loss.detach())
            optimizer.step()
            optimizer.zero_grad()
            if self.frustum_feature_selection:
                for key, val in c.items():
                    if (self.coarse_mapper and "coarse" in key) or (not self.coarse_mapper and "coarse" not in key):
                        vg, mask = masked[key]
                        val = val.detach()
                        val[mask] = vg.detach()
                        c[key] = val

        for p, rg in saved_rg.items():
            p.requires_grad_(rg)
        if not self.BA:
            return None
        cam_id = 0
        for frame in optimize_frame:
            if frame != -1:
                if frame != oldest_frame:
                    c2w = get_camera_from_tensor(cam_tensors[cam_id].detach())
                    keyframe_dict[frame]["est_c2w"] = torch.cat([c2w, bottom], 0).clone()
                    cam_id += 1
            else:
                c2w = get_camera_from_tensor(cam_tensors[-1].detach())
                cur_c2w = torch.cat([c2w, bottom], 0).clone()
        return cur_c2w
