"""GPU tests of the Tracker / Mapper drop-ins against an oracle-driven replica of the same loop.

Pixel selection is random in the reference (torch.randint, common.py:99); both sides here consume
the same pre-drawn pixel indices (select_uv is monkeypatched), so the loops are comparable.
Checked: Tracker.optimize_cam_in_batch loss + camera gradient + Adam update (src/Tracker.py:71-128);
Mapper.optimize_map per-iteration losses over the middle → fine → colour schedule and the
first-iteration grid gradients (src/Mapper.py:230-540).
"""
import copy
import importlib
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from conftest import FixedPixels, grids_from, rel_l2, sd_from
from oracle import nslam_oracle as orc

pytestmark = pytest.mark.gpu
P = importlib.import_module("nice-slam_amd")


def base_cfg():
    return {
        "coarse": False, "occupancy": True, "scale": 1,
        "rendering": {"N_samples": 32, "N_surface": 16, "N_importance": 0, "lindisp": False, "perturb": 0.0},
        "tracking": {"lr": 0.001, "device": "cuda:0", "iters": 3, "gt_camera": False, "pixels": 200,
                     "seperate_LR": False, "w_color_loss": 0.5, "ignore_edge_W": 20, "ignore_edge_H": 20,
                     "handle_dynamic": True, "use_color_in_tracking": True, "const_speed_assumption": True},
        "mapping": {"device": "cuda:0", "fix_fine": True, "BA_cam_lr": 0.001, "fix_color": False, "pixels": 400,
                    "iters": 5, "w_color_loss": 0.2, "fine_iter_ratio": 0.6, "middle_iter_ratio": 0.4,
                    "mapping_window_size": 5, "frustum_feature_selection": False,
                    "keyframe_selection_method": "overlap",
                    "stage": {"middle": {"decoders_lr": 0.0, "coarse_lr": 0.0, "middle_lr": 0.1, "fine_lr": 0.0,
                                         "color_lr": 0.0},
                              "fine": {"decoders_lr": 0.0, "coarse_lr": 0.0, "middle_lr": 0.005, "fine_lr": 0.005,
                                       "color_lr": 0.0},
                              "color": {"decoders_lr": 0.005, "coarse_lr": 0.0, "middle_lr": 0.005,
                                        "fine_lr": 0.005, "color_lr": 0.005}}},
    }


class Scene:
    def __init__(self, tiny, H=96, W=128):
        self.dev = torch.device("cuda:0")
        self.bound = torch.from_numpy(tiny["bound"])
        self.sd = sd_from(tiny)
        self.grids = {k: v for k, v in grids_from(tiny).items() if k != "grid_coarse"}
        self.H, self.W, self.fx, self.fy = H, W, 60.0, 60.0
        self.cx, self.cy = (W - 1) / 2, (H - 1) / 2
        c2w = torch.from_numpy(tiny["c2w"]).float()
        self.c2w = c2w
        g = torch.Generator().manual_seed(3)
        jj, ii = torch.meshgrid(torch.arange(H, dtype=torch.float32), torch.arange(W, dtype=torch.float32),
                                indexing="ij")
        ro, rd = orc.rays_from_uv(ii.reshape(-1), jj.reshape(-1), c2w, self.fx, self.fy, self.cx, self.cy)
        far = orc.far_bound(ro, rd, self.bound).float()
        self.depth = (far * (0.6 + 0.3 * torch.rand(far.shape, generator=g))).reshape(H, W)
        self.depth[torch.rand(H, W, generator=g) < 0.05] = 0
        self.color = torch.rand(H, W, 3, generator=g)

    def slam(self, cfg):
        nice = P.NICE(c_dim=32, coarse=False, middle_grid_len=0.64, fine_grid_len=0.32, color_grid_len=0.32)
        nice.load_state_dict({k: v.clone() for k, v in self.sd.items() if not k.startswith("coarse")})
        nice.set_bound(self.bound)
        s = SimpleNamespace(nice=True, bound=self.bound, H=self.H, W=self.W, fx=self.fx, fy=self.fy, cx=self.cx,
                            cy=self.cy, shared_decoders=nice.to(self.dev),
                            shared_c={k: v.to(self.dev).contiguous(memory_format=torch.channels_last_3d)
                                      for k, v in self.grids.items()},
                            estimate_c2w_list=torch.zeros(4, 4, 4), gt_c2w_list=torch.zeros(4, 4, 4),
                            mapping_idx=torch.zeros(1).int())
        s.renderer = P.Renderer(cfg, None, s)
        return s


def oracle_samples(scene, idx, H0, H1, W0, W1, c2w, depth, color):
    jj, ii = torch.meshgrid(torch.arange(H0, H1, dtype=torch.float32), torch.arange(W0, W1, dtype=torch.float32),
                            indexing="ij")
    i, j = ii.reshape(-1)[idx], jj.reshape(-1)[idx]
    ro, rd = orc.rays_from_uv(i, j, c2w, scene.fx, scene.fy, scene.cx, scene.cy)
    return ro, rd, depth[H0:H1, W0:W1].reshape(-1)[idx], color[H0:H1, W0:W1].reshape(-1, 3)[idx]


def test_tracker_optimize_cam_in_batch(tiny, monkeypatch):
    sc = Scene(tiny)
    cfg = base_cfg()
    fp = FixedPixels()
    monkeypatch.setattr(P.common, "select_uv", fp)
    tr = P.Tracker(cfg, None, sc.slam(cfg))
    tr.update_para_from_mapping()
    cam0 = P.common.get_tensor_from_camera(sc.c2w).cuda()
    cam = cam0.clone().requires_grad_(True)
    opt = torch.optim.Adam([cam], lr=0.001)
    losses = [tr.optimize_cam_in_batch(cam, sc.color.cuda(), sc.depth.cuda(), 200, opt) for _ in range(3)]
    # oracle replica
    camo = cam0.cpu().clone().requires_grad_(True)
    opto = torch.optim.Adam([camo], lr=0.001)
    ref_losses = []
    for k in range(3):
        opto.zero_grad()
        c2w = orc.camera_from_tensor(camo)
        ro, rd, gd, gc = oracle_samples(sc, fp.log[k], 20, sc.H - 20, 20, sc.W - 20, c2w, sc.depth, sc.color)
        keep = orc.inside_mask(ro, rd, gd, sc.bound)
        ro, rd, gd, gc = ro[keep], rd[keep], gd[keep], gc[keep]
        d, v, c = orc.render_batch_ray(sc.sd, sc.grids, rd, ro, "color", sc.bound, gd)
        loss = orc.tracker_loss(d, v, c, gd, gc)
        loss.backward()
        opto.step()
        ref_losses.append(float(loss))
    np.testing.assert_allclose(losses, ref_losses, rtol=2e-4)
    assert rel_l2(cam.detach().cpu().numpy() - cam0.cpu().numpy(),
                  camo.detach().numpy() - cam0.cpu().numpy()) < 1e-2


def test_mapper_optimize_map_schedule(tiny, monkeypatch):
    sc = Scene(tiny)
    cfg = base_cfg()
    fp = FixedPixels(seed=5)
    monkeypatch.setattr(P.common, "select_uv", fp)
    slam = sc.slam(cfg)
    mp_ = P.Mapper(cfg, None, slam)
    mp_.loss_history = []
    kf = [{"gt_c2w": sc.c2w, "idx": 0, "color": sc.color, "depth": sc.depth, "est_c2w": sc.c2w.clone()}]
    out = mp_.optimize_map(5, 1.0, 1, sc.color, sc.depth, sc.c2w, kf, [0], sc.c2w.clone())
    assert out is None
    losses = [float(x) for x in mp_.loss_history]
    # oracle replica of optimize_map with frustum_feature_selection=False, BA=False
    sd = {k: v.clone() for k, v in sc.sd.items() if not k.startswith("coarse")}
    for k in sd:
        if k.startswith("color_decoder."):
            sd[k].requires_grad_(True)
    grids = {k: v.clone().requires_grad_(True) for k, v in sc.grids.items()}
    st = cfg["mapping"]["stage"]
    groups = [[v for k, v in sd.items() if k.startswith("color_decoder.")], [], [grids["grid_middle"]],
              [grids["grid_fine"]], [grids["grid_color"]]]
    opt = torch.optim.Adam([{"params": g, "lr": 0} for g in groups])
    ref, n = [], 5
    for it in range(n):
        stage = "middle" if it <= int(n * 0.4) else ("fine" if it <= int(n * 0.6) else "color")
        for gi, name in enumerate(("decoders", "coarse", "middle", "fine", "color")):
            opt.param_groups[gi]["lr"] = st[stage][name + "_lr"]
        opt.zero_grad()
        # draw 0 is the overlap keyframe selection's (Mapper.py:185-186); then 2 frames per iteration
        parts = [oracle_samples(sc, fp.log[1 + 2 * it + f], 0, sc.H, 0, sc.W, sc.c2w, sc.depth, sc.color)
                 for f in range(2)]
        ro, rd, gd, gc = (torch.cat([p[q] for p in parts]) for q in range(4))
        keep = orc.inside_mask(ro, rd, gd, sc.bound)
        ro, rd, gd, gc = ro[keep], rd[keep], gd[keep], gc[keep]
        d, v, c = orc.render_batch_ray(sd, grids, rd, ro, stage, sc.bound, gd)
        loss = orc.mapper_loss(d, c, gd, gc, stage)
        loss.backward()
        opt.step()
        ref.append(float(loss))
    np.testing.assert_allclose(losses, ref, rtol=2e-3)
    for k in grids:
        delta = slam.shared_c[k].detach().cpu() - sc.grids[k]
        rdelta = grids[k].detach() - sc.grids[k]
        # measured on MI355X: middle 1.7e-5, fine 3.9e-4, colour 5.1e-5
        assert rel_l2(delta.numpy(), rdelta.numpy()) < 5e-3, k


def _nudged(c2w, ang, t):
    """c2w rotated by `ang` rad about z and shifted by t: a distinct keyframe pose."""
    ca, sa = float(np.cos(ang)), float(np.sin(ang))
    R = torch.tensor([[ca, -sa, 0.0], [sa, ca, 0.0], [0.0, 0.0, 1.0]], dtype=torch.float32)
    out = c2w.clone()
    out[:3, :3] = R @ c2w[:3, :3]
    out[:3, 3] += torch.tensor(t, dtype=torch.float32)
    return out


def test_mapper_bundle_adjustment(tiny, monkeypatch):
    """BA on (the ScanNet config, BASELINE configs[2]): the camera 7-vectors of every window frame
    but the oldest get gradients through the rays (Mapper.py:346-363, 441-448) and an Adam step at
    BA_cam_lr in the colour stage (Mapper.py:420-421); optimize_map returns the updated current pose
    and writes the keyframes' est_c2w back (Mapper.py:520-540)."""
    sc = Scene(tiny)
    cfg = base_cfg()
    fp = FixedPixels(seed=9)
    monkeypatch.setattr(P.common, "select_uv", fp)
    slam = sc.slam(cfg)
    mp_ = P.Mapper(cfg, None, slam)
    mp_.BA = True
    mp_.loss_history = []
    monkeypatch.setattr(mp_, "keyframe_selection_overlap", lambda *a, **k: [0])
    est = [sc.c2w.clone(), _nudged(sc.c2w, 0.01, (0.01, -0.005, 0.0))]
    cur = _nudged(sc.c2w, -0.008, (0.0, 0.006, 0.004))
    kf = [{"gt_c2w": sc.c2w, "idx": i, "color": sc.color, "depth": sc.depth, "est_c2w": est[i].clone()}
          for i in range(2)]
    n = 5
    out = mp_.optimize_map(n, 1.0, 2, sc.color, sc.depth, sc.c2w, kf, [0, 1], cur.clone())
    assert out is not None and tuple(out.shape) == (4, 4)
    losses = [float(x) for x in mp_.loss_history]

    # oracle replica: window [0, 1, -1]; the oldest frame (0) stays fixed, frames 1 and -1 are optimised
    sd = {k: v.clone() for k, v in sc.sd.items() if not k.startswith("coarse")}
    for k in sd:
        if k.startswith("color_decoder."):
            sd[k].requires_grad_(True)
    grids = {k: v.clone().requires_grad_(True) for k, v in sc.grids.items()}
    cams = [P.common.get_tensor_from_camera(est[1]).cpu().float().requires_grad_(True),
            P.common.get_tensor_from_camera(cur).cpu().float().requires_grad_(True)]
    st = cfg["mapping"]["stage"]
    groups = [[v for k, v in sd.items() if k.startswith("color_decoder.")], [], [grids["grid_middle"]],
              [grids["grid_fine"]], [grids["grid_color"]], cams]
    opt = torch.optim.Adam([{"params": g, "lr": 0} for g in groups])
    ref = []
    for it in range(n):
        stage = "middle" if it <= int(n * 0.4) else ("fine" if it <= int(n * 0.6) else "color")
        for gi, name in enumerate(("decoders", "coarse", "middle", "fine", "color")):
            opt.param_groups[gi]["lr"] = st[stage][name + "_lr"]
        if stage == "color":
            opt.param_groups[5]["lr"] = cfg["mapping"]["BA_cam_lr"]
        opt.zero_grad()
        poses = [est[0], orc.camera_from_tensor(cams[0]), orc.camera_from_tensor(cams[1])]
        parts = [oracle_samples(sc, fp.log[3 * it + f], 0, sc.H, 0, sc.W, poses[f], sc.depth, sc.color)
                 for f in range(3)]
        ro, rd, gd, gc = (torch.cat([p[q] for p in parts]) for q in range(4))
        keep = orc.inside_mask(ro, rd, gd, sc.bound)
        ro, rd, gd, gc = ro[keep], rd[keep], gd[keep], gc[keep]
        d, v, c = orc.render_batch_ray(sd, grids, rd, ro, stage, sc.bound, gd)
        loss = orc.mapper_loss(d, c, gd, gc, stage)
        loss.backward()
        opt.step()
        ref.append(float(loss))
    np.testing.assert_allclose(losses, ref, rtol=2e-3)
    # compare poses (q and -q are the same rotation): the update each camera received
    for got, cam, start in ((kf[1]["est_c2w"], cams[0], est[1]), (out, cams[1], cur)):
        ref_pose = orc.camera_from_tensor(cam.detach())
        d_got = got[:3].detach().cpu() - start[:3]
        d_ref = ref_pose - start[:3]
        assert float(d_ref.abs().max()) > 1e-5  # the colour-stage step moved the camera
        # the step is Adam's m/sqrt(v) over five camera gradients (lr 0 until the colour stage) whose
        # components change sign between iterations: the cancellation in m amplifies the run-to-run float
        # atomics order of the grid updates before it — 8.2e-5 typical, 1.3e-3 seen once on MI355X (the
        # d/dpts kernel itself is bit-identical across builds, tools/probes/pg_equal.py)
        assert rel_l2(d_got.numpy(), d_ref.numpy()) < 5e-3
    assert torch.equal(kf[0]["est_c2w"], est[0])  # the oldest frame is not optimised
