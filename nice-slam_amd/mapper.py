"""Mapper drop-in: map optimisation on the HIP render path (src/Mapper.py).

`optimize_map` keeps the reference's signature and semantics (Mapper.py:230-540): staged
middle → fine → colour schedule, Adam re-created per call, frustum-masked grid parameters,
optional bundle adjustment of keyframe cameras.  It runs on the fused mapping engine
(engine.MappingEngine: one gather / sampler / forward / loss / backward / Adam chain of HIP launches
per iteration, no autograd) — `Mapper.fused = False` selects the autograd drop-in of the same loop.
Differences from the reference (none changes the maths):
  * keyframe images stay resident on the device (the reference copies them host→device every
    iteration, Mapper.py:439-440);
  * the frustum voxel mask (Mapper.py:93-164) is computed with torch on the device; cv2.remap's
    bilinear lookup is emulated including its 1/32-pixel fixed-point positions and zero border
    (OpenCV is not installed: parity with cv2 itself is unpinned);
  * the masked grid vectors are not copied in and out of the grids every iteration
    (Mapper.py:394-401, 511-519): Adam updates the selected voxels in place, with state for them
    alone — the same elementwise update; the optimiser's state is reset per call (a fresh Adam);
  * the inside-mask prefilter (Mapper.py:469-481) gives dropped rays zero loss weight instead of
    compacting them (their gradients are exactly zero; the sampler's batch max sees kept rays only);
  * pixel draws: through common.select_uv (torch.randint, eager) when it is replaced (tests pin the
    draws that way) or a generator is given; otherwise drawn inside the gather kernel (uniform over
    the image like select_uv, a counter-based stream instead of torch's Philox) so that each stage's
    iterations are captured ONCE in a hipGraph and replayed by every later call of the same shape
    (the window's frames are copied into persistent slots, the frustum selection is bound on the
    device with capacity-sized buffers: engine.MappingEngine.bind_masks).
The mapping loop driver (Mapper.run, Mapper.py:542-657) is out of scope (dataset/meshing/ckpt glue).
"""
from __future__ import annotations

import numpy as np
import torch

from . import common as _common
from . import ops
from .common import get_camera_from_tensor, get_samples, get_tensor_from_camera, random_select

_SELECT_UV = _common.select_uv  # the product's own pixel selection (a replacement one forces eager draws)
_STAGE_GROUPS = ("decoders", "coarse", "middle", "fine", "color")


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


_KMAT = {}


def _intrinsics(fx, fy, cx, cy, dev):
    """The camera matrix as a float64 device tensor, made once per (intrinsics, device): a hipGraph
    capturing its users must not copy it from the host."""
    key = (float(fx), float(fy), float(cx), float(cy), str(dev))
    if key not in _KMAT:
        _KMAT[key] = torch.tensor([[fx, 0.0, cx], [0.0, fy, cy], [0.0, 0.0, 1.0]], dtype=torch.float64, device=dev)
    return _KMAT[key]


_POINTS = {}


def _grid_points(bound, val_shape, dev):
    """The grid's voxel positions in get_mask_from_c2w's meshgrid order [X*Y*Z, 3] (cached per shape)."""
    b = bound
    key = (tuple(float(v) for v in torch.as_tensor(b).reshape(-1)), tuple(int(v) for v in val_shape), str(dev))
    if key not in _POINTS:
        nz, ny, nx = (int(v) for v in val_shape)
        X, Y, Z = torch.meshgrid(torch.linspace(float(b[0][0]), float(b[0][1]), nx, device=dev),
                                 torch.linspace(float(b[1][0]), float(b[1][1]), ny, device=dev),
                                 torch.linspace(float(b[2][0]), float(b[2][1]), nz, device=dev), indexing="ij")
        _POINTS[key] = torch.stack([X, Y, Z], dim=-1).reshape(-1, 3)
    return _POINTS[key]


def frustum_rows_device(c2w, val_shape, depth, bound, H, W, fx, fy, cx, cy, slot, rows, n_live, mask_ref=None):
    """frustum_mask fused with its compaction (ABI v20 nslam_frustum_rows): slot [Z*Y*X] int32, rows (>= the
    voxel count) int32 and n_live int64 [1] are written in place, as MappingEngine.bind_masks would from the
    mask.  The two projection GEMMs and the near-camera test run here with frustum_mask's own torch ops (the
    same values bit for bit); the remap, the depth tests and the compaction run in one kernel sequence.
    mask_ref: optional uint8 [X*Y*Z] receiving the mask in frustum_mask's order."""
    from ._lib import check, lib, ptr, stream_ptr
    dev = depth.device
    points = _grid_points(bound, val_shape, dev)
    c2w = c2w.to(dev).float()
    w2c = torch.linalg.inv_ex(c2w)[0]
    cam = points @ w2c[:3, :3].T + w2c[:3, 3]
    cam = cam.double()
    cam[:, 0] *= -1
    uvz = cam @ _intrinsics(fx, fy, cx, cy, dev).T
    d = points - c2w[:3, 3]
    near = ((d * d).sum(1) < 0.5 * 0.5).to(torch.uint8)
    nz, ny, nx = (int(v) for v in val_shape)
    n = nx * ny * nz
    wsb = lib().nslam_frustum_rows_workspace_size(n)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    dep = depth.float().contiguous()
    rc = lib().nslam_frustum_rows(ptr(uvz.contiguous()), ptr(near), ptr(dep), H, W, nx, ny, nz, ptr(slot), ptr(rows),
                                  ptr(n_live), ptr(mask_ref), ptr(ws), wsb, stream_ptr(dev))
    check(rc, "nslam_frustum_rows")


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
    w2c = torch.linalg.inv_ex(c2w)[0]  # (torch.linalg.inv without its error check: no host sync, capturable)
    cam = points @ w2c[:3, :3].T + w2c[:3, 3]
    cam = cam.double()
    cam[:, 0] *= -1
    K = _intrinsics(fx, fy, cx, cy, dev)
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
        self.fused = True   # optimize_map on engine.MappingEngine (False: the autograd drop-in)
        self.graphs = True  # fused path with device draws: each stage's iterations as one cached hipGraph
        self._eng = None
        self._fopt = None
        self._cam = {}      # number of BA cameras -> (cams, grad, ws, tickets, FusedAdam)
        self._slots = None  # (depth [F,H,W], color [F,H,W,3], c2w [F,4,4]) of the window
        self._setup = None  # persistent inputs of the captured per-call setup (_setup_inputs)
        self._graphs = {}
        # the device draws' stream key (from torch's CPU generator, so torch.manual_seed pins it)
        self._draw_seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        self.calls = 0
        self.timing = None  # set to [] to record per-call phase times (host clock + HIP events; bench legs)

    # ------------------------------------------------------------------------------------------
    def get_mask_from_c2w(self, c2w, key, val_shape, depth):
        """Frustum voxel selection (Mapper.py:93-164) → bool mask [X, Y, Z] on the device."""
        return frustum_mask(c2w, key, val_shape, depth, self.bound, self.H, self.W, self.fx, self.fy, self.cx,
                            self.cy)

    def keyframe_overlap_scores(self, gt_color, gt_depth, c2w, keyframe_dict, N_samples=16, pixels=100):
        """Mapper.py:185-221: per keyframe, the fraction of the current frame's near-surface samples
        (100 pixels × 16 depths in [0.8·d, d + 0.5]) that project inside it (20-px margin, in front
        of the camera).  One host sync for all keyframes (the reference's loop is host numpy)."""
        counts, n = self._overlap_counts(gt_color, gt_depth, c2w, [kf["est_c2w"] for kf in keyframe_dict], N_samples,
                                         pixels)
        if counts is None:
            return []
        # mask.sum() / uv.shape[0] as the reference divides: an integer count over the sample count
        return [int(cnt) / n for cnt in counts.cpu()]

    def _overlap_counts(self, gt_color, gt_depth, c2w, poses, N_samples=16, pixels=100):
        """The device half of keyframe_overlap_scores: (counts [len(poses)] device int64 or None, samples)."""
        dev = self.device
        H, W, fx, fy, cx, cy = self.H, self.W, self.fx, self.fy, self.cx, self.cy
        rays_o, rays_d, gd, _ = get_samples(0, H, 0, W, pixels, H, W, fx, fy, cx, cy, c2w, gt_depth, gt_color, dev,
                                            generator=self.generator)
        if not poses:
            return None, 0
        gd = gd.reshape(-1, 1).repeat(1, N_samples)
        t = torch.linspace(0.0, 1.0, N_samples, device=dev)
        z = gd * 0.8 * (1.0 - t) + (gd + 0.5) * t
        verts = (rays_o[..., None, :] + rays_d[..., None, :] * z[..., :, None]).reshape(-1, 3)
        K = _intrinsics(fx, fy, cx, cy, dev)
        counts = []
        for pose in poses:
            w2c = torch.linalg.inv_ex(pose.to(dev).float())[0]
            cam = (verts @ w2c[:3, :3].T + w2c[:3, 3]).double()
            cam[:, 0] *= -1
            uvz = cam @ K.T
            zz = uvz[:, 2] + 1e-5
            uv = (uvz[:, :2] / zz[:, None]).float()
            edge = 20
            m = (uv[:, 0] < W - edge) & (uv[:, 0] > edge) & (uv[:, 1] < H - edge) & (uv[:, 1] > edge) & (zz < 0)
            counts.append(m.sum())
        return torch.stack(counts), verts.shape[0]

    def keyframe_selection_overlap(self, gt_color, gt_depth, c2w, keyframe_dict, k, N_samples=16, pixels=100):
        """Mapper.py:166-228: keyframes whose frustum sees the current frame's surface samples,
        ranked by overlap (stable sort, as `sorted`), then a random permutation (numpy RNG) of the
        ones with any overlap, truncated to k."""
        scores = self.keyframe_overlap_scores(gt_color, gt_depth, c2w, keyframe_dict, N_samples, pixels)
        return self._rank_keyframes(scores, k)

    @staticmethod
    def _rank_keyframes(scores, k):
        """The host half of keyframe_selection_overlap (Mapper.py:222-228)."""
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
        self.calls += 1
        if self.fused:
            return self._optimize_map_fused(num_joint_iters, lr_factor, idx, cur_gt_color, cur_gt_depth, gt_cur_c2w,
                                            keyframe_dict, keyframe_list, cur_c2w)
        return self._optimize_map_autograd(num_joint_iters, lr_factor, idx, cur_gt_color, cur_gt_depth, gt_cur_c2w,
                                           keyframe_dict, keyframe_list, cur_c2w)

    # ------------------------------------------------------------------------------------------
    def _select_window(self, keyframe_dict, keyframe_list, cur_gt_color, cur_gt_depth, cur_c2w):
        """optimize_frame (keyframe ids, -1 = the current frame) and the oldest one (Mapper.py:256-272,
        346-349)."""
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
        return optimize_frame, oldest_frame

    def _stage_of(self, joint_iter, num_joint_iters):
        """Mapper.py:403-411."""
        if self.coarse_mapper:
            return "coarse"
        if joint_iter <= int(num_joint_iters * self.middle_iter_ratio):
            return "middle"
        if joint_iter <= int(num_joint_iters * self.fine_iter_ratio):
            return "fine"
        return "color"

    def _grid_keys(self):
        return ["grid_coarse"] if self.coarse_mapper else [k for k in ("grid_middle", "grid_fine", "grid_color")
                                                          if k in self.c]

    def engine(self):
        """The persistent MappingEngine over the shared grids and decoders (built on first use)."""
        if self._eng is None:
            from .engine import MappingEngine
            c = {k: self.c[k] for k in self._grid_keys()}
            r = self.renderer
            self._eng = MappingEngine(self.decoders, c, self.bound, r.N_samples, r.N_surface, lindisp=r.lindisp,
                                      w_color=self.w_color_loss, device=self.device)
        return self._eng

    def _trainable(self):
        """Decoders in the optimiser's "decoders" group (Mapper.py:335-341)."""
        return tuple(n for n, fixed in (("fine", self.fix_fine), ("color", self.fix_color)) if not fixed)

    def _optimizer(self, eng):
        """The persistent FusedAdam of the fused path: groups decoders / coarse / middle / fine / colour as
        the reference's (Mapper.py:365-389); grid groups hold the frustum rows with their live count."""
        if self._fopt is None:
            dec = [eng.decs[n].param for n in self._trainable() if n in eng.decs]
            groups = [{"params": dec, "lr": 0.0}]
            for name in _STAGE_GROUPS[1:]:
                k = "grid_" + name
                if k in eng.c:
                    rows, n_live = eng.live_rows(k)
                    groups.append({"params": [eng.c[k]], "lr": 0.0, "rows": rows, "n_live": n_live})
                else:
                    groups.append({"params": [], "lr": 0.0})
            self._fopt = ops.FusedAdam(groups)
        return self._fopt

    def _cam_state(self, n):
        """Persistent BA camera buffers for n cameras: cams [n,7], their gradient, the camera-gradient
        workspace / tickets, and their Adam (the reference's param group 5, Mapper.py:386-389)."""
        if n not in self._cam:
            dev = self.device
            cams = torch.zeros(n, 7, dtype=torch.float32, device=dev)
            grad = torch.zeros(n, 7, dtype=torch.float32, device=dev)
            ws = torch.zeros(n * ops.CAM_GRAD_WS_DOUBLES, dtype=torch.float64, device=dev)
            tickets = torch.zeros(n, dtype=torch.int32, device=dev)
            self._cam[n] = (cams, grad, ws, tickets, ops.FusedAdam([{"params": [cams], "lr": 0.0}]))
        return self._cam[n]

    def _window_slots(self, F):
        if self._slots is None or self._slots[0].shape[0] < F:
            dev, H, W = self.device, self.H, self.W
            n = max(F, self.mapping_window_size)
            self._slots = (torch.zeros(n, H, W, dtype=torch.float32, device=dev),
                           torch.zeros(n, H, W, 3, dtype=torch.float32, device=dev),
                           torch.eye(4, dtype=torch.float32, device=dev).repeat(n, 1, 1))
            self._graphs.clear()  # (captured against the old slots)
        return self._slots

    def _bind_frustum(self, eng, c2w, depth):
        """This call's frustum selection bound into the engine's capacity buffers (Mapper.py:314-333): the
        fused kernel (nslam_frustum_rows) per grid shape, the other grids of that shape copying its rows;
        the coarse grid (an all-true mask, Mapper.py:113-115) and frustum_feature_selection=False through
        bind_masks.  get_mask_from_c2w replaced on the instance (a test hook) also goes through bind_masks."""
        keys = self._grid_keys()
        if (not self.frustum_feature_selection or self.coarse_mapper
                or "get_mask_from_c2w" in self.__dict__):
            eng.bind_masks(self._call_masks(c2w, depth))
            return
        if getattr(eng, "_cap_keys", None) != tuple(sorted(keys)):
            eng.bind_masks({k: None for k in keys})  # (first call: the capacity buffers)
        done = {}
        for k in keys:
            shp = tuple(self.c[k].shape[2:])
            rows, n_live = eng.live_rows(k)
            slot = eng.slot[k]
            if shp in done:
                s0, r0, n0 = done[shp]
                slot.copy_(s0)
                rows.copy_(r0)
                n_live.copy_(n0)
            else:
                frustum_rows_device(c2w, shp, depth, self.bound, self.H, self.W, self.fx, self.fy, self.cx, self.cy,
                                    slot, rows, n_live)
                done[shp] = (slot, rows, n_live)

    def _call_masks(self, c2w, depth):
        """This call's frustum masks (Mapper.py:314-333; None = every voxel): grids of one shape share one."""
        masks, by_shape = {}, {}
        for k in self._grid_keys():
            shp = tuple(self.c[k].shape[2:])
            if not self.frustum_feature_selection:
                masks[k] = None
            elif k == "grid_coarse":
                masks[k] = self.get_mask_from_c2w(c2w, k, shp, depth)
            else:
                if shp not in by_shape:
                    by_shape[shp] = self.get_mask_from_c2w(c2w, k, shp, depth)
                masks[k] = by_shape[shp]
        return masks

    def _setup_inputs(self, K):
        """Persistent inputs of the captured per-call setup: the current frame, its pose, the keyframe poses."""
        st = self._setup
        if st is None or st["poses"].shape[0] < K:
            dev, H, W = self.device, self.H, self.W
            st = self._setup = {"depth": torch.zeros(H, W, dtype=torch.float32, device=dev),
                                "color": torch.zeros(H, W, 3, dtype=torch.float32, device=dev),
                                "c2w": torch.eye(4, dtype=torch.float32, device=dev),
                                "poses": torch.eye(4, dtype=torch.float32, device=dev).repeat(max(8, 2 * K), 1, 1)}
            self._graphs = {k: v for k, v in self._graphs.items() if k[0] != "setup"}  # (bound to the old buffers)
        return st

    def _optimize_map_fused(self, num_joint_iters, lr_factor, idx, cur_gt_color, cur_gt_depth, gt_cur_c2w,
                            keyframe_dict, keyframe_list, cur_c2w):
        """optimize_map on the fused engine (see the module docstring)."""
        dev = self.device
        H, W = self.H, self.W
        tm = None
        if self.timing is not None:
            import time
            tm = {"t0": time.perf_counter(), "clock": time.perf_counter, "ev": {}}

        def mark(name):  # host time and a HIP event on the caller's stream at a phase boundary
            if tm is not None:
                tm[name] = tm["clock"]()
                e = torch.cuda.Event(enable_timing=True)
                e.record()
                tm["ev"][name] = e

        cur_gt_depth = cur_gt_depth.to(dev).float()
        cur_gt_color = cur_gt_color.to(dev).float()
        cur_c2w = cur_c2w.to(dev).float()
        eng = self.engine()
        for d in eng.decs.values():  # parameters may have been assigned since the last call
            d.repack()
        device_draws = _common.select_uv is _SELECT_UV and self.generator is None
        use_graphs = self.graphs and device_draws
        # Everything that does not depend on the keyframe selection is enqueued first: the selection reads
        # its overlap scores back to the host (the reference's numpy ranking), and what is queued before
        # that read overlaps the previous call's iterations still running on the device: this call's
        # frustum selection (Mapper.py:314-333) bound on the device, a fresh Adam (Mapper.py:365-389: zero
        # moments and step counts) and, with graphs, the overlap counts — one captured graph per keyframe count.
        overlap_here = (use_graphs and self.keyframe_selection_method == "overlap" and len(keyframe_dict) > 1
                        and "keyframe_selection_overlap" not in self.__dict__)
        if use_graphs:
            kfs = keyframe_dict[:-1] if overlap_here else []
            st = self._setup_inputs(len(kfs))
            st["depth"].copy_(cur_gt_depth)
            st["color"].copy_(cur_gt_color)
            st["c2w"][:cur_c2w.shape[0]].copy_(cur_c2w)
            if kfs:
                st["poses"][:len(kfs)].copy_(torch.stack([kf["est_c2w"].to(dev).float()[:4] for kf in kfs]))

            def setup():
                self._bind_frustum(eng, st["c2w"], st["depth"])
                o = self._optimizer(eng)
                o.init_state()
                o.reset_state()
                if kfs:
                    cnt, n = self._overlap_counts(st["color"], st["depth"], st["c2w"],
                                                  [st["poses"][i] for i in range(len(kfs))])
                    return cnt, n
                return None, 0

            key = ("setup", len(kfs))
            if key not in self._graphs:
                setup()  # eager warm-up: first-time allocations (engine capacity buffers, Adam state, caches)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    out = setup()
                self._graphs[key] = (g, out)
            g, (counts, n_samp) = self._graphs[key]
            g.replay()
            opt = self._optimizer(eng)
        else:
            self._bind_frustum(eng, cur_c2w, cur_gt_depth)
            opt = self._optimizer(eng)
            opt.reset_state()
        mark("masks")
        if overlap_here:  # the window from the captured overlap counts (one read-back; Mapper.py:256-272)
            scores = [int(c) / n_samp for c in counts.cpu()]
            optimize_frame = self._rank_keyframes(scores, self.mapping_window_size - 2)
            oldest_frame = None
            if len(keyframe_list) > 0:
                optimize_frame = optimize_frame + [len(keyframe_list) - 1]
                oldest_frame = min(optimize_frame)
            optimize_frame += [-1]
        else:
            optimize_frame, oldest_frame = self._select_window(keyframe_dict, keyframe_list, cur_gt_color,
                                                               cur_gt_depth, cur_c2w)
        mark("selected")
        F = len(optimize_frame)
        n_per = self.mapping_pixels // F
        # window slots: the oldest frame (fixed under BA) first, then the others in optimize_frame order
        order = list(optimize_frame)
        if self.BA and oldest_frame is not None:
            order.remove(oldest_frame)
            order.insert(0, oldest_frame)
        depth_s, color_s, c2w_s = self._window_slots(F)
        poses = []
        for s, fr in enumerate(order):
            if fr == -1:
                d, c, m = cur_gt_depth, cur_gt_color, cur_c2w
            else:
                d, c = self._frame_images(keyframe_dict[fr])
                m = keyframe_dict[fr]["est_c2w"].to(dev).float()
            depth_s[s].copy_(d)
            color_s[s].copy_(c)
            poses.append(m[:3])
        poses = torch.stack(poses)
        c2w_s[:F, :3].copy_(poses)
        frames = [(depth_s[s], color_s[s], c2w_s[s]) for s in range(F)]
        c0 = 1 if (self.BA and oldest_frame is not None) else 0
        ncam = (F - c0) if self.BA else 0
        cam = None
        if ncam:  # the 7-vectors of the optimised frames (Mapper.py:349-363)
            cams, cgrad, cws, ctk, copt = cam = self._cam_state(ncam)
            copt.init_state()

            def cams_init():  # (captured with the first stage's graph below)
                ops.cam_vector_batch(c2w_s[c0:F], cams)  # get_tensor_from_camera of each, one launch
                copt.reset_state()

            # the optimised frames are gathered from their 7-vectors: the gather forms each pose
            # (get_camera_from_tensor) and writes it to the frame's slot for the camera gradient (ABI v21)
            frames[c0:] = [(depth_s[s], color_s[s], c2w_s[s], cams[s - c0]) for s in range(c0, F)]

        def post_bwd(gps, ro, rd, z):  # BA: camera gradients of every optimised frame, then their Adam step
            ops.cam_grad_batch(cams, c2w_s[c0:F], [(c0 + k) * n_per for k in range(ncam)], n_per, gps, z, rd, cgrad,
                               cws, ctk)
            copt.step(grads={cams: cgrad})

        intr = (self.fx, self.fy, self.cx, self.cy)
        tdec = self._trainable()
        ar = torch.arange(H * W, device=dev) if not device_draws else None
        # device draws: the next iteration's gather + sampler run beside this one's render and backward
        # (engine prefetch); every run of one stage starts with its own batch (eng._pre reset), so a
        # captured run holds its whole prefetch chain.  With BA the poses the rays come from move only in
        # the colour stage (the cameras' lr is 0 before it, Mapper.py:420-421: their Adam state advances,
        # the 7-vectors do not), so only colour-stage BA iterations draw their rays serially.
        def prefetch_for(stage):
            return device_draws and (not ncam or stage != "color")

        def iteration(stage, record=None):
            pix = None
            if not device_draws:  # select_uv per frame, in optimize_frame order (Mapper.py:437-467)
                pix = torch.empty(F * n_per, dtype=torch.int64, device=dev)
                for fr in optimize_frame:
                    s = order.index(fr)
                    pix[s * n_per:(s + 1) * n_per] = _common.select_uv(ar, ar, n_per, ar, ar.view(-1, 1).expand(-1, 3),
                                                                       device=dev, generator=self.generator)[0]
            ray_loss, _ = eng.iteration(stage, frames, pix, n_per, (H, W), intr, opt, trainable_decoders=tdec,
                                        use_gt_in_sampler=not self.coarse_mapper, seed=self._draw_seed,
                                        post_bwd=post_bwd if ncam else None, prefetch=prefetch_for(stage))
            if record is not None:
                record(ray_loss)

        def set_lr(stage, zero=False):
            st_ = self.cfg["mapping"]["stage"][stage]
            for gi, name in enumerate(_STAGE_GROUPS):
                opt.param_groups[gi]["lr"] = 0.0 if zero else st_[name + "_lr"] * lr_factor
            if cam is not None:
                copt.param_groups[0]["lr"] = self.BA_cam_lr if (stage == "color" and not zero) else 0.0

        # the call's schedule as runs of one stage (Mapper.py:403-421)
        runs = []
        for it in range(num_joint_iters):
            stg = self._stage_of(it, num_joint_iters)
            if runs and runs[-1][0] == stg:
                runs[-1][1] += 1
            else:
                runs.append([stg, 1])
        hist = self.loss_history
        plan = []
        warmed = False
        if use_graphs:
            # the warm-up iterations below draw pixels too: the draw stream is rewound afterwards, so a call
            # draws the same pixels whether its graphs were cached or just captured (and as the eager path)
            ctr = eng.draws(self._draw_seed).counter
            ctr0 = ctr.clone()
            for ri, (stg, n) in enumerate(runs):
                first = ri == 0 and ncam > 0  # the first run's graph also sets the BA cameras up
                key = ("stage", stg, n, F, n_per, c0, ncam, float(lr_factor), hist is not None, tdec, first)
                if key not in self._graphs:
                    # one zero-lr eager iteration (the maps do not move; lazily made streams, events, tickets
                    # and draw counters exist before capture), then the capture itself (nothing runs)
                    if ncam:
                        cams_init()
                    set_lr(stg, zero=True)
                    eng._pre = None
                    iteration(stg)
                    warmed = True
                    set_lr(stg)
                    losses = torch.zeros(n, dtype=torch.float64, device=dev) if hist is not None else None
                    g = torch.cuda.CUDAGraph()
                    eng._pre = None
                    with torch.cuda.graph(g, capture_error_mode="thread_local"):
                        if first:
                            cams_init()
                        for i in range(n):
                            iteration(stg, None if losses is None else (lambda rl, i=i: losses[i].copy_(rl.sum())))
                    self._graphs[key] = (g, losses)
                plan.append((stg, n, self._graphs[key]))
            ctr.copy_(ctr0)
        if warmed:  # (the warm-up steps moved the Adam state and rewrote the BA cameras' poses)
            opt.reset_state()
            c2w_s[:F, :3].copy_(poses)
        mark("window")
        if use_graphs:
            for stg, n, (g, losses) in plan:
                self.stage = stg
                g.replay()
                if hist is not None:
                    hist.extend(losses.clone().unbind())
        else:
            if ncam:
                cams_init()
            for stg, n in runs:
                self.stage = stg
                set_lr(stg)
                eng._pre = None
                for _ in range(n):
                    iteration(stg, None if hist is None else (lambda rl: hist.append(rl.sum())))
        mark("iterations")
        if tm is not None:
            self.timing.append(tm)
        if not ncam:
            return None
        # BA write-back (Mapper.py:521-540): the optimised poses of the keyframes and the current frame
        out = torch.zeros(ncam, 4, 4, dtype=torch.float32, device=dev)
        out[:, 3, 3] = 1.0
        ops.cam_pose_batch(cams, out)
        for k in range(ncam):
            fr = order[c0 + k]
            if fr == -1:
                cur_c2w = out[k]
            else:
                keyframe_dict[fr]["est_c2w"] = out[k]
        return cur_c2w

    def _optimize_map_autograd(self, num_joint_iters, lr_factor, idx, cur_gt_color, cur_gt_depth, gt_cur_c2w,
                               keyframe_dict, keyframe_list, cur_c2w):
        """The autograd drop-in of optimize_map (Mapper.py:230-540 line for line, HIP ops under autograd)."""
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
