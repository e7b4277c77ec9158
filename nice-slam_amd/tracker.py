"""Tracker drop-in: camera optimisation on the HIP render path (src/Tracker.py).

`optimize_cam_in_batch` keeps the reference's signature and semantics (Tracker.py:71-128).
The frame loop's per-frame logic (Tracker.py:184-256) is `track_frame`; dataset loading,
process synchronisation and visualisation (Tracker.py:144-183) are out of scope.
"""
from __future__ import annotations

import copy

import numpy as np
import torch

from . import common as _common
from .common import camera_tensors, get_camera_from_tensor, get_samples, get_tensor_from_camera

_SELECT_UV = _common.select_uv


class Tracker(object):
    def __init__(self, cfg, args, slam, generator=None):
        self.cfg = cfg
        self.args = args
        self.scale = cfg.get("scale", 1)
        self.coarse = cfg["coarse"]
        self.occupancy = cfg["occupancy"]
        self.nice = slam.nice
        self.bound = slam.bound
        self.renderer = slam.renderer
        self.shared_c = slam.shared_c
        self.shared_decoders = slam.shared_decoders
        self.estimate_c2w_list = slam.estimate_c2w_list
        self.gt_c2w_list = slam.gt_c2w_list
        self.mapping_idx = slam.mapping_idx
        t = cfg["tracking"]
        self.cam_lr = t["lr"]
        self.device = t["device"]
        self.num_cam_iters = t["iters"]
        self.gt_camera = t["gt_camera"]
        self.tracking_pixels = t["pixels"]
        self.seperate_LR = t["seperate_LR"]
        self.w_color_loss = t["w_color_loss"]
        self.ignore_edge_W = t["ignore_edge_W"]
        self.ignore_edge_H = t["ignore_edge_H"]
        self.handle_dynamic = t["handle_dynamic"]
        self.use_color_in_tracking = t["use_color_in_tracking"]
        self.const_speed_assumption = t["const_speed_assumption"]
        self.H, self.W, self.fx, self.fy, self.cx, self.cy = slam.H, slam.W, slam.fx, slam.fy, slam.cx, slam.cy
        self.prev_mapping_idx = -1
        self.generator = generator  # pixel-selection RNG (None = torch's global device generator)
        self.c = {}
        self.decoders = None
        self._bound_dev = None
        self.fused = True     # track_frame on engine.TrackingEngine (no host sync per iteration)
        self.graphs = True    # fused, no generator: a frame's camera loop is one cached hipGraph (device draws)
        self._engine = None
        self._fstate = None   # persistent buffers of the captured camera loop
        self._graphs = {}
        self._draw_seed = int(torch.randint(0, 2 ** 62, (1,)).item())

    def _inside_mask(self, rays_o, rays_d, gt_depth):
        """Tracker.py:95-100: keep rays whose AABB exit distance >= gt depth."""
        if self._bound_dev is None or self._bound_dev.device != rays_o.device:
            self._bound_dev = self.bound.to(rays_o.device)
        with torch.no_grad():
            t = (self._bound_dev.unsqueeze(0) - rays_o.detach().unsqueeze(-1)) / rays_d.detach().unsqueeze(-1)
            t, _ = torch.min(torch.max(t, dim=2)[0], dim=1)
            return t >= gt_depth

    def optimize_cam_in_batch(self, camera_tensor, gt_color, gt_depth, batch_size, optimizer):
        """One camera iteration: sample pixels, render, uncertainty-weighted L1, backward, step."""
        device = self.device
        H, W, fx, fy, cx, cy = self.H, self.W, self.fx, self.fy, self.cx, self.cy
        optimizer.zero_grad()
        c2w = get_camera_from_tensor(camera_tensor)
        Wedge, Hedge = self.ignore_edge_W, self.ignore_edge_H
        rays_o, rays_d, b_depth, b_color = get_samples(Hedge, H - Hedge, Wedge, W - Wedge, batch_size, H, W, fx, fy,
                                                       cx, cy, c2w, gt_depth, gt_color, device,
                                                       generator=self.generator)
        if self.nice:
            keep = self._inside_mask(rays_o, rays_d, b_depth)
            rays_d, rays_o, b_depth, b_color = rays_d[keep], rays_o[keep], b_depth[keep], b_color[keep]
        depth, uncertainty, color = self.renderer.render_batch_ray(self.c, self.decoders, rays_d, rays_o, device,
                                                                   stage="color", gt_depth=b_depth)
        uncertainty = uncertainty.detach()
        resid = torch.abs(b_depth - depth) / torch.sqrt(uncertainty + 1e-10)
        if self.handle_dynamic:
            mask = (resid < 10 * resid.median()) & (b_depth > 0)
        else:
            mask = b_depth > 0
        loss = resid[mask].sum()
        if self.use_color_in_tracking:
            loss = loss + self.w_color_loss * torch.abs(b_color - color)[mask].sum()
        loss.backward()
        optimizer.step()
        optimizer.zero_grad()
        return loss.item()

    def update_para_from_mapping(self):
        """Tracker.py:130-142: snapshot the mapper's decoders and grids (no gradients needed).  The first
        snapshot is a deep copy; later ones are copied into it in place, so the tracking engine (and the
        hipGraphs captured over it) stay bound to the same buffers."""
        if self.mapping_idx[0] != self.prev_mapping_idx:
            same = (self.decoders is not None and set(self.c) == set(self.shared_c)
                    and all(self.c[k].shape == v.shape and self.c[k].stride() == v.stride()
                            for k, v in self.shared_c.items()))
            if same:
                with torch.no_grad():
                    for a, b in zip(self.decoders.parameters(), self.shared_decoders.parameters()):
                        a.copy_(b)
                    for key, val in self.shared_c.items():
                        self.c[key].copy_(val)
                if self._engine is not None:
                    for d in self._engine.eng.decs.values():  # the MFMA-packed copies of the new weights
                        d.repack()
            else:
                self.decoders = copy.deepcopy(self.shared_decoders).to(self.device)
                # tracking optimises the camera only: decoder/grid gradients are never used
                self.decoders.requires_grad_(False)
                for key, val in self.shared_c.items():
                    self.c[key] = val.detach().clone().to(self.device)
                self._engine = None  # re-bound to the new snapshot on first use
                self._fstate = None
                self._graphs.clear()
            self.prev_mapping_idx = self.mapping_idx[0].clone()

    def engine(self):
        """TrackingEngine over the current decoder/grid snapshot."""
        if self._engine is None:
            from .engine import TrackingEngine
            from .ops import channels_last
            r = self.renderer
            c = {k: channels_last(v) for k, v in self.c.items() if k != "grid_coarse"}
            self._engine = TrackingEngine(self.decoders, c, self.bound, r.N_samples, r.N_surface, (self.H, self.W),
                                          (self.fx, self.fy, self.cx, self.cy),
                                          ignore_edge=(self.ignore_edge_H, self.ignore_edge_W),
                                          w_color=self.w_color_loss, handle_dynamic=self.handle_dynamic,
                                          use_color=self.use_color_in_tracking, device=self.device)
        return self._engine

    def track_frame(self, idx, gt_color, gt_depth, gt_c2w, pre_c2w=None, prev2_c2w=None):
        """Per-frame camera estimate (Tracker.py:184-256, without sync/visualisation) → c2w [4,4]."""
        device = self.device
        self.update_para_from_mapping()
        gt_depth, gt_color = gt_depth.to(device), gt_color.to(device)
        if idx == 0 or self.gt_camera:
            return gt_c2w.clone()
        if (self.fused and self.graphs and not self.seperate_LR and self.generator is None
                and _common.select_uv is _SELECT_UV):
            return self._track_graph(gt_color, gt_depth, pre_c2w,
                                     prev2_c2w if self.const_speed_assumption else None)
        if self.const_speed_assumption and prev2_c2w is not None:
            pre = pre_c2w.float().to(device)
            delta = pre @ torch.linalg.inv_ex(prev2_c2w.to(device).float())[0]  # (no error check: no sync)
            est = delta @ pre
        else:
            est = pre_c2w.to(device)
        # (on the device: no host round trip per frame)
        camera_tensor = camera_tensors(est.detach().float()[None])[0] if self.fused else \
            get_tensor_from_camera(est.detach()).to(device)
        if self.seperate_LR:
            T = camera_tensor[-3:].clone().requires_grad_(True)
            quad = camera_tensor[:4].clone().requires_grad_(True)
            optimizer = torch.optim.Adam([{"params": [T], "lr": self.cam_lr},
                                          {"params": [quad], "lr": self.cam_lr * 0.2}])
        else:
            camera_tensor = camera_tensor.clone().requires_grad_(True)
            optimizer = torch.optim.Adam([camera_tensor], lr=self.cam_lr)
        best, best_loss = None, np.inf
        if self.fused and not self.seperate_LR:
            return self._track_fused(camera_tensor, gt_color, gt_depth)
        for _ in range(self.num_cam_iters):
            if self.seperate_LR:
                camera_tensor = torch.cat([quad, T], 0)
            loss = self.optimize_cam_in_batch(camera_tensor, gt_color, gt_depth, self.tracking_pixels, optimizer)
            if loss < best_loss:
                best_loss, best = loss, camera_tensor.clone().detach()
        bottom = torch.tensor([[0, 0, 0, 1.0]], dtype=torch.float32, device=device)
        return torch.cat([get_camera_from_tensor(best), bottom], 0)

    def _track_fused(self, camera_tensor, gt_color, gt_depth):
        """The camera loop of track_frame (Tracker.py:225-250) on the TrackingEngine: the best pose
        (lowest pre-step loss → the pose right after that step, as the reference keeps it) is
        selected on the device; no host sync.  Without a generator the pixels are drawn in the gather
        kernel and the whole loop is ONE hipGraph, captured on the first frame and replayed on every
        later one (the frame is copied into persistent slots; a fresh Adam per frame by resetting its
        state).  With a generator (pinned draws): torch.randint per iteration, eager."""
        from .ops import FusedAdam
        eng = self.engine()
        device = self.device
        cam = camera_tensor.detach().clone().requires_grad_(True)
        opt = FusedAdam([{"params": [cam], "lr": self.cam_lr}])
        best = cam.detach().clone()
        best_loss = torch.full((), float("inf"), dtype=torch.float64, device=device)
        depth = gt_depth.float().contiguous()
        color = gt_color.float().contiguous()
        for _ in range(self.num_cam_iters):
            pix = torch.randint(eng.n_window(), (self.tracking_pixels,), device=device, generator=self.generator)
            eng.iteration(cam, depth, color, pix, opt, best=(best_loss, best))  # (+ Tracker.py:245-247)
        bottom = torch.tensor([[0, 0, 0, 1.0]], dtype=torch.float32, device=device)
        return torch.cat([get_camera_from_tensor(best), bottom], 0)

    def _track_graph(self, gt_color, gt_depth, pre_c2w, prev2_c2w):
        """track_frame's whole per-frame work as ONE captured hipGraph, replayed for every frame: the pose
        guess (constant speed, Tracker.py:191-198), its camera 7-vector, a fresh Adam, the camera loop with
        device pixel draws and the device-side best-pose selection (Tracker.py:225-250), and the result pose.
        Per frame the host copies the frame and the previous poses into persistent buffers and replays."""
        from . import ops
        from .ops import FusedAdam
        eng = self.engine()
        dev = self.device
        st = self._fstate
        if st is None:
            cam = torch.zeros(7, dtype=torch.float32, device=dev).requires_grad_(True)
            out = torch.eye(4, dtype=torch.float32, device=dev)
            st = self._fstate = {
                "depth": torch.zeros(self.H, self.W, dtype=torch.float32, device=dev),
                "color": torch.zeros(self.H, self.W, 3, dtype=torch.float32, device=dev),
                "pre": torch.eye(4, dtype=torch.float32, device=dev), "prev2": torch.eye(4, dtype=torch.float32, device=dev),
                "cam": cam, "opt": FusedAdam([{"params": [cam], "lr": self.cam_lr}]),
                "best": torch.zeros(7, dtype=torch.float32, device=dev),
                "best_loss": torch.zeros((), dtype=torch.float64, device=dev), "out": out}
            st["opt"].init_state()
        cam, opt, best, best_loss = st["cam"], st["opt"], st["best"], st["best_loss"]
        st["depth"].copy_(gt_depth)
        st["color"].copy_(gt_color)
        st["pre"][:3].copy_(pre_c2w[:3])  # (the bottom row stays [0, 0, 0, 1])
        speed = prev2_c2w is not None
        if speed:
            st["prev2"][:3].copy_(prev2_c2w[:3])
        n, iters = self.tracking_pixels, self.num_cam_iters

        def frame(zero_lr=False):
            pre = st["pre"]
            est = (pre @ torch.linalg.inv_ex(st["prev2"])[0]) @ pre if speed else pre
            # the guess's 7-vector into the camera and the best pose in one launch (ABI v22)
            ops.cam_vector_batch(est[None], cam.detach().view(1, 7), best.view(1, 7))
            best_loss.fill_(float("inf"))
            opt.reset_state()
            for _ in range(1 if zero_lr else iters):
                # (the iteration's loss launch also keeps the best pose, Tracker.py:245-247)
                eng.iteration(cam, st["depth"], st["color"], None, opt, n=n, seed=self._draw_seed,
                              best=(best_loss, best))
            ops.cam_pose(best, st["out"][:3])  # get_camera_from_tensor(best), one launch

        key = (iters, n, speed)
        if key not in self._graphs:
            # one zero-lr eager iteration (camera grad, Adam ticket, draw counter, caches made before capture);
            # the draw stream is rewound, so the frame draws as it would have eagerly
            ctr = eng.eng.draws(self._draw_seed).counter
            ctr0 = ctr.clone()
            opt.param_groups[0]["lr"] = 0.0
            frame(zero_lr=True)
            opt.param_groups[0]["lr"] = self.cam_lr
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                frame()
            self._graphs[key] = g
            ctr.copy_(ctr0)
        self._graphs[key].replay()
        return st["out"].clone()
