"""Golden vectors for the LOOP-level pieces of the path, produced by the reference's own code
(build container only; the .npz it writes is what the tests read on the GPU box).

Run:  PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_loop.py

Cases (reference file:line they execute):
  camera      get_camera_from_tensor / quad2rotation (common.py:137-176), get_rays_from_uv
              (common.py:74-89) and pts = o + d·z (Renderer.py:172-174): poses and the VJP to the
              7-vector for fixed d loss/d pts.
  tloss       Tracker.optimize_cam_in_batch's loss (Tracker.py:110-125) on fixed raw / z: loss and
              d loss / d raw through raw2outputs_nerf_color (common.py:204-245).
  mloss_*     Mapper.optimize_map's loss (Mapper.py:487-503), colour and middle stage, likewise.
  track       Tracker.optimize_cam_in_batch (Tracker.py:71-128), 3 iterations on the tiny scene:
              losses, camera gradients, cameras after each Adam step.
  map         Mapper.optimize_map (Mapper.py:230-540) with frustum feature selection, overlap
              keyframe selection and bundle adjustment over a 5-frame window (BASELINE configs[2]):
              per-iteration losses, selected frames, grids / colour decoder / poses after the call.
  frustum     Mapper.get_mask_from_c2w (Mapper.py:93-164) at Replica room0 grid shapes.
  overlap     Mapper.keyframe_selection_overlap (Mapper.py:166-228) at room0 shapes: the
              per-keyframe percent_inside scores and the selection.

Harness (nothing of the reference is copied or modified; it is imported and called):
  * src.Tracker / src.Mapper import cv2 and colorama at module level, and neither is installed.
    Stand-in modules are registered first: colorama's Fore / Style (print colours only) and
    cv2.remap — the only cv2 call on these paths (Mapper.py:134-137) — as a numpy restatement
    of OpenCV's INTER_LINEAR / BORDER_CONSTANT remap with 1/32-pixel fixed-point positions.
    The frustum masks are therefore pinned to the reference's code around that lookup; parity
    of the lookup with OpenCV itself stays unpinned.
  * quad2rotation places its output with .to(quad.get_device()) (common.py:150), which is -1 on
    CPU: while the reference runs here, Tensor.get_device reports "cpu" for CPU tensors.
  * get_tensor_from_camera needs Blender's mathutils (absent): Mapper's bundle-adjustment camera
    tensors are made by `quat_from_c2w` below (standard rotation → quaternion, w >= 0).
  * select_uv's torch.randint is replaced by `FixedDraws` (a seeded CPU generator, logged) so the
    drop-ins draw the same pixels; np.random is seeded before the keyframe permutation.
  * loss values are read by wrapping torch.Tensor.backward for the duration of a call; the
    overlap scores by wrapping the `sorted` the Mapper module calls.
  * NICE.forward builds 'cuda:N' for the non-colour stages (decoder.py:316): the mapper runs on
    `StageCombiner` (make_golden.py), which applies the stage combiner over the reference
    sub-decoders.
"""
import contextlib
import os
import sys
import types
from types import SimpleNamespace

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import scenes  # noqa: E402
from make_golden import StageCombiner, ref_nice, ref_renderer  # noqa: E402

from oracle import nslam_oracle as orc  # noqa: E402


# ------------------------------------------------------------------------------------------------
# stand-in modules for the two uninstalled imports
# ------------------------------------------------------------------------------------------------
def remap_linear(img, map_x, map_y):
    """cv2.remap(img, map_x, map_y, INTER_LINEAR) for float32 maps, BORDER_CONSTANT (0):
    position rounded to 1/32 pixel (cvRound), taps outside the image read 0, weights
    (1-fy)(1-fx), fx(1-fy), (1-fx)fy, fx·fy in float32, summed in tap order."""
    img = np.asarray(img, dtype=np.float32)
    H, W = img.shape[:2]
    mx = np.asarray(map_x, dtype=np.float32).reshape(-1)
    my = np.asarray(map_y, dtype=np.float32).reshape(-1)
    X = np.rint(np.clip(mx.astype(np.float64) * 32, -2 ** 31, 2 ** 31 - 1)).astype(np.int64)
    Y = np.rint(np.clip(my.astype(np.float64) * 32, -2 ** 31, 2 ** 31 - 1)).astype(np.int64)
    x0, y0 = X >> 5, Y >> 5
    fx = (X & 31).astype(np.float32) / np.float32(32)
    fy = (Y & 31).astype(np.float32) / np.float32(32)

    def tap(x, y):
        ok = (x >= 0) & (x < W) & (y >= 0) & (y < H)
        return np.where(ok, img[np.clip(y, 0, H - 1), np.clip(x, 0, W - 1)], np.float32(0))

    one = np.float32(1)
    out = (tap(x0, y0) * ((one - fy) * (one - fx)) + tap(x0 + 1, y0) * ((one - fy) * fx)
           + tap(x0, y0 + 1) * (fy * (one - fx)) + tap(x0 + 1, y0 + 1) * (fy * fx))
    return out.astype(np.float32).reshape(-1, 1)


def _install_stubs():
    cv2 = types.ModuleType("cv2")
    cv2.INTER_LINEAR = 1

    def remap(src, map1, map2, interpolation=1, **kw):
        assert interpolation == 1
        return remap_linear(src, map1, map2)

    cv2.remap = remap
    sys.modules.setdefault("cv2", cv2)
    colorama = types.ModuleType("colorama")
    colorama.Fore = SimpleNamespace(CYAN="", RED="", GREEN="", YELLOW="", BLUE="", MAGENTA="", WHITE="", RESET="")
    colorama.Style = SimpleNamespace(RESET_ALL="", BRIGHT="")
    sys.modules.setdefault("colorama", colorama)


_install_stubs()
import src.common as ref_common  # noqa: E402  (reference)
import src.Mapper as ref_mapper_mod  # noqa: E402  (reference)
import src.Tracker as ref_tracker_mod  # noqa: E402  (reference)
from src.common import get_camera_from_tensor, get_rays_from_uv, raw2outputs_nerf_color  # noqa: E402

torch.set_num_threads(8)


@contextlib.contextmanager
def cpu_get_device():
    """quad2rotation's .to(quad.get_device()) (common.py:150) on CPU tensors."""
    orig = torch.Tensor.get_device

    def gd(self):
        d = orig(self)
        return "cpu" if d == -1 else d

    torch.Tensor.get_device = gd
    try:
        yield
    finally:
        torch.Tensor.get_device = orig


@contextlib.contextmanager
def record_losses(out):
    orig = torch.Tensor.backward

    def bw(self, *a, **k):
        out.append(float(self.detach()))
        return orig(self, *a, **k)

    torch.Tensor.backward = bw
    try:
        yield
    finally:
        torch.Tensor.backward = orig


class FixedDraws:
    """select_uv (common.py:92-107) with a seeded CPU generator; logs every draw."""

    def __init__(self, seed):
        self.g = torch.Generator().manual_seed(seed)
        self.log = []

    def __call__(self, i, j, n, depth, color, device="cuda:0", generator=None):
        i, j = i.reshape(-1), j.reshape(-1)
        idx = torch.randint(i.shape[0], (n,), generator=self.g)
        self.log.append(idx.clone())
        return i[idx], j[idx], depth.reshape(-1)[idx], color.reshape(-1, 3)[idx]


@contextlib.contextmanager
def fixed_draws(seed):
    fd = FixedDraws(seed)
    orig = ref_common.select_uv
    ref_common.select_uv = fd
    try:
        yield fd
    finally:
        ref_common.select_uv = orig


def quat_from_c2w(RT):
    """Rotation → quaternion (w, x, y, z), w >= 0, + translation (stand-in for mathutils'
    Matrix.to_quaternion in get_tensor_from_camera, common.py:179-201)."""
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
    return torch.from_numpy(np.concatenate([q, T])).float()


def tiny_inputs():
    with np.load(os.path.join(HERE, "tiny_scene.npz")) as z:
        tiny = {k: z[k] for k in z.files}
    bound = torch.from_numpy(tiny["bound"])
    b2, _, _ = scenes.tiny_window()
    assert np.array_equal(b2, tiny["bound"]), (b2, tiny["bound"])
    sd = {k[3:]: torch.from_numpy(v) for k, v in tiny.items() if k.startswith("sd.")}
    grids = {k: torch.from_numpy(tiny[k]) for k in ("grid_middle", "grid_fine", "grid_color")}
    return bound, sd, grids


# ------------------------------------------------------------------------------------------------
def camera_case(gen):
    """get_camera_from_tensor + rays + pts and the VJP to the 7-vector (common.py:74-89,137-176)."""
    out = {}
    B, n, S = 16, 40, 16
    cams = torch.randn(B, 7, generator=gen)
    cams[:8, :4] = cams[:8, :4] / cams[:8, :4].norm(dim=1, keepdim=True)   # unit quaternions too
    cams[:, 4:] *= 2.0
    cam = SimpleNamespace(**scenes.ROOM0_CAM)
    i = torch.rand(B, n, generator=gen) * cam.W
    j = torch.rand(B, n, generator=gen) * cam.H
    z = torch.rand(B, n, S, generator=gen, dtype=torch.float64) * 5
    gp = torch.randn(B, n, S, 3, generator=gen, dtype=torch.float64)
    c2ws, rds, grads = [], [], []
    with cpu_get_device():
        for b in range(B):
            t = cams[b].clone().requires_grad_(True)
            c2w = get_camera_from_tensor(t)
            ro, rd = get_rays_from_uv(i[b], j[b], c2w, cam.H, cam.W, cam.fx, cam.fy, cam.cx, cam.cy, "cpu")
            pts = ro[..., None, :] + rd[..., None, :] * z[b][..., :, None]   # Renderer.py:172-174
            (g,) = torch.autograd.grad(pts, (t,), gp[b])
            c2ws.append(c2w.detach())
            rds.append(rd.detach())
            grads.append(g)
    out.update({"cam": cams, "i": i, "j": j, "z": z, "g_pts": gp, "c2w": torch.stack(c2ws),
                "rays_d": torch.stack(rds), "grad_cam": torch.stack(grads)})
    return out


class FixedRawRenderer:
    """render_batch_ray stand-in: composites a fixed raw / z with the reference compositing, so
    the reference's loss code is what turns them into a loss and d loss / d raw."""

    def __init__(self, raw, z):
        self.raw = raw.clone().requires_grad_(True)
        self.z = z
        self.seen = {}

    def render_batch_ray(self, c, decoders, rays_d, rays_o, device, stage, gt_depth=None):
        assert rays_d.shape[0] == self.raw.shape[0], (rays_d.shape, self.raw.shape)
        self.seen = {"gt_depth": None if gt_depth is None else gt_depth.detach().clone(), "stage": stage,
                     "rays_d": rays_d.detach().clone()}
        depth, unc, color, _ = raw2outputs_nerf_color(self.raw * 1.0, self.z, rays_d, occupancy=True, device="cpu")
        return depth, unc, color


def _loss_scene(gen, n, S, cam):
    """Pose inside a big box and depths well inside it, so every ray passes the inside-mask."""
    bound = torch.tensor([[-50.0, 50.0], [-50.0, 50.0], [-50.0, 50.0]], dtype=torch.float64)
    c2w = torch.from_numpy(scenes.look_pose([0.0, 0.0, 0.0], 0.3, 0.2))
    depth = (torch.rand(cam.H, cam.W, generator=gen) * 3 + 0.5).float()
    depth[torch.rand(cam.H, cam.W, generator=gen) < 0.08] = 0.0
    color = torch.rand(cam.H, cam.W, 3, generator=gen)
    raw = torch.randn(n, S, 4, generator=gen) * 0.5
    z = torch.sort(torch.rand(n, S, generator=gen, dtype=torch.float64) * 4, -1).values
    return bound, c2w, depth, color, raw, z


def tracker_loss_case(gen, handle_dynamic):
    cam = SimpleNamespace(H=60, W=80, fx=50.0, fy=50.0, cx=39.5, cy=29.5)
    n, S = 300, 48
    bound, c2w, depth, color, raw, z = _loss_scene(gen, n, S, cam)
    # a few far-off depths: the handle_dynamic median mask (Tracker.py:111-113) drops them
    raw[:12, :, 3] = 8.0
    rnd = FixedRawRenderer(raw, z)
    tr = object.__new__(ref_tracker_mod.Tracker)
    tr.__dict__.update(device="cpu", H=cam.H, W=cam.W, fx=cam.fx, fy=cam.fy, cx=cam.cx, cy=cam.cy, ignore_edge_W=20,
                       ignore_edge_H=20, nice=True, bound=bound, renderer=rnd, c={}, decoders=None,
                       handle_dynamic=handle_dynamic, use_color_in_tracking=True, w_color_loss=0.5)
    camt = quat_from_c2w(c2w).requires_grad_(True)
    opt = torch.optim.Adam([camt], lr=0.001)
    with cpu_get_device(), fixed_draws(21) as fd:
        loss = tr.optimize_cam_in_batch(camt, color, depth, n, opt)
    idx = fd.log[0]
    win_d = depth[20:cam.H - 20, 20:cam.W - 20].reshape(-1)[idx]
    win_c = color[20:cam.H - 20, 20:cam.W - 20].reshape(-1, 3)[idx]
    assert torch.equal(rnd.seen["gt_depth"], win_d)
    return {"raw": raw, "z": z, "gt_depth": win_d, "gt_color": win_c, "loss": np.float64(loss),
            "g_raw": rnd.raw.grad.detach()}


def mapper_loss_case(gen, stage):
    cam = SimpleNamespace(H=60, W=80, fx=50.0, fy=50.0, cx=39.5, cy=29.5)
    n, S = 400, 48
    bound, c2w, depth, color, raw, z = _loss_scene(gen, n, S, cam)
    rnd = FixedRawRenderer(raw, z)
    mp = object.__new__(ref_mapper_mod.Mapper)
    ratio = 0.4 if stage == "middle" else -1.0   # joint_iter 0 <= int(1*ratio): middle; -1: colour
    mp.__dict__.update(_mapper_attrs(cam, bound, rnd, None, {}, pixels=n, frustum=False, window=5,
                                     middle_ratio=ratio, fine_ratio=ratio, fix_color=True))
    mp.BA = False
    losses = []
    with fixed_draws(22) as fd, record_losses(losses):
        mp.optimize_map(1, 1.0, 3, color, depth, c2w, [], [], torch.cat([c2w, torch.tensor([[0, 0, 0, 1.0]])])
                        if c2w.shape[0] == 3 else c2w)
    assert rnd.seen["stage"] == stage, rnd.seen["stage"]
    idx = fd.log[0]
    return {"raw": raw, "z": z, "gt_depth": depth.reshape(-1)[idx], "gt_color": color.reshape(-1, 3)[idx],
            "loss": np.float64(losses[0]), "g_raw": rnd.raw.grad.detach()}


def _mapper_attrs(cam, bound, renderer, decoders, c, pixels, frustum, window, middle_ratio=0.4, fine_ratio=0.6,
                  fix_color=False):
    stage = {"coarse": {"decoders_lr": 0.0, "coarse_lr": 0.001, "middle_lr": 0.0, "fine_lr": 0.0, "color_lr": 0.0},
             "middle": {"decoders_lr": 0.0, "coarse_lr": 0.0, "middle_lr": 0.1, "fine_lr": 0.0, "color_lr": 0.0},
             "fine": {"decoders_lr": 0.0, "coarse_lr": 0.0, "middle_lr": 0.005, "fine_lr": 0.005, "color_lr": 0.0},
             "color": {"decoders_lr": 0.005, "coarse_lr": 0.0, "middle_lr": 0.005, "fine_lr": 0.005,
                       "color_lr": 0.005}}   # configs/nice_slam.yaml:70-95
    return dict(H=cam.H, W=cam.W, fx=cam.fx, fy=cam.fy, cx=cam.cx, cy=cam.cy, c=c, cfg={"mapping": {"stage": stage}},
                device="cpu", keyframe_selection_method="overlap", mapping_window_size=window, keyframe_dict=[],
                save_selected_keyframes_info=False, mapping_pixels=pixels, nice=True,
                frustum_feature_selection=frustum, fix_fine=True, fix_color=fix_color, decoders=decoders,
                coarse_mapper=False, middle_iter_ratio=middle_ratio, fine_iter_ratio=fine_ratio, BA_cam_lr=0.001,
                no_vis_on_first_frame=True, output="Demo", renderer=renderer, w_color_loss=0.2, occupancy=True,
                bound=bound, stage="middle")


def tracker_loop_case():
    bound, sd, grids = tiny_inputs()
    cam = SimpleNamespace(**scenes.TINY_CAM)
    b, poses, cur = scenes.tiny_window()
    c2w = torch.from_numpy(cur)
    depth = torch.from_numpy(scenes.box_depth(cur, scenes.TINY_CAM, b, seed=40))
    color = torch.from_numpy(scenes.color_image(scenes.TINY_CAM, seed=41))
    m = ref_nice(sd, bound)
    r = ref_renderer(bound)
    r.H, r.W, r.fx, r.fy, r.cx, r.cy = cam.H, cam.W, cam.fx, cam.fy, cam.cx, cam.cy
    tr = object.__new__(ref_tracker_mod.Tracker)
    tr.__dict__.update(device="cpu", H=cam.H, W=cam.W, fx=cam.fx, fy=cam.fy, cx=cam.cx, cy=cam.cy, ignore_edge_W=20,
                       ignore_edge_H=20, nice=True, bound=bound, renderer=r, c={k: v.clone() for k, v in grids.items()},
                       decoders=m, handle_dynamic=True, use_color_in_tracking=True, w_color_loss=0.5)
    # a perturbed start pose, as the constant-speed guess gives (Tracker.py:191-198)
    start = c2w.clone()
    start[:3, 3] += torch.tensor([0.03, -0.02, 0.015])
    cam0 = quat_from_c2w(start)
    camt = cam0.clone().requires_grad_(True)
    opt = torch.optim.Adam([camt], lr=0.001)
    grads, cams, losses = [], [], []
    step = opt.step

    def step_rec(*a, **k):
        grads.append(camt.grad.detach().clone())
        return step(*a, **k)

    opt.step = step_rec
    with cpu_get_device(), fixed_draws(23):
        for _ in range(3):
            losses.append(tr.optimize_cam_in_batch(camt, color, depth, 200, opt))
            cams.append(camt.detach().clone())
    return {"cam0": cam0, "losses": np.asarray(losses), "grads": torch.stack(grads), "cams": torch.stack(cams),
            "depth_seed": np.int64(40), "color_seed": np.int64(41), "draw_seed": np.int64(23)}


def mapper_loop_case():
    bound, sd, grids = tiny_inputs()
    cam = SimpleNamespace(**scenes.TINY_CAM)
    b, poses, cur = scenes.tiny_window()
    m = ref_nice(sd, bound)
    comb = StageCombiner(m)
    comb.fine_decoder, comb.color_decoder = m.fine_decoder, m.color_decoder
    r = ref_renderer(bound)
    c = {k: v.clone() for k, v in grids.items()}
    kf = []
    for k, p in enumerate(poses):
        kf.append({"gt_c2w": torch.from_numpy(p), "idx": 5 * k, "est_c2w": torch.from_numpy(p).clone(),
                   "depth": torch.from_numpy(scenes.box_depth(p, scenes.TINY_CAM, b, seed=100 + k)),
                   "color": torch.from_numpy(scenes.color_image(scenes.TINY_CAM, seed=200 + k))})
    kf_list = [5 * k for k in range(len(poses))]
    cur_depth = torch.from_numpy(scenes.box_depth(cur, scenes.TINY_CAM, b, seed=150))
    cur_color = torch.from_numpy(scenes.color_image(scenes.TINY_CAM, seed=250))
    mp = object.__new__(ref_mapper_mod.Mapper)
    mp.__dict__.update(_mapper_attrs(cam, bound, r, comb, c, pixels=1000, frustum=True, window=5))
    mp.BA = True
    sel = []
    orig_sel = mp.keyframe_selection_overlap

    def sel_rec(*a, **k):
        out = orig_sel(*a, **k)
        sel.append(list(out))
        return out

    mp.keyframe_selection_overlap = sel_rec
    orig_q = ref_mapper_mod.get_tensor_from_camera
    ref_mapper_mod.get_tensor_from_camera = quat_from_c2w
    n_iters = 8
    losses = []
    masks = {}
    orig_mask = mp.get_mask_from_c2w

    def mask_rec(c2w, key, val_shape, depth_np):
        mk = orig_mask(c2w, key, val_shape, depth_np)
        masks[key] = np.asarray(mk).copy()
        return mk

    mp.get_mask_from_c2w = mask_rec
    np.random.seed(7)
    try:
        with cpu_get_device(), fixed_draws(24), record_losses(losses):
            out_c2w = mp.optimize_map(n_iters, 1.0, 30, cur_color, cur_depth, torch.from_numpy(cur), kf, kf_list,
                                      torch.from_numpy(cur).clone())
    finally:
        ref_mapper_mod.get_tensor_from_camera = orig_q
    res = {"n_iters": np.int64(n_iters), "losses": np.asarray(losses), "selected": np.asarray(sel[0], dtype=np.int64),
           "np_seed": np.int64(7), "draw_seed": np.int64(24), "cur_c2w_out": out_c2w.detach()}
    for k in range(len(poses)):
        res[f"est_c2w_out.{k}"] = kf[k]["est_c2w"].detach()
    for k, v in c.items():
        res["grid_out." + k] = v.detach()
        res["mask." + k] = masks[k]
    for k, v in m.color_decoder.state_dict().items():
        res["color_decoder_out." + k] = v.detach()
    return res


def frustum_case():
    b, poses, cur = scenes.room0_window()
    cam = SimpleNamespace(**scenes.ROOM0_CAM)
    mp = object.__new__(ref_mapper_mod.Mapper)
    mp.__dict__.update(H=cam.H, W=cam.W, fx=cam.fx, fy=cam.fy, cx=cam.cx, cy=cam.cy,
                       bound=torch.from_numpy(b))
    depth = scenes.box_depth(cur, scenes.ROOM0_CAM, b, seed=300)
    lens = {"grid_middle": 0.32, "grid_fine": 0.16, "grid_color": 0.16}
    out = {"depth_seed": np.int64(300)}
    for key, gl in lens.items():
        shp = orc.grid_shape(torch.from_numpy(b), gl)[2:]
        mk = mp.get_mask_from_c2w(torch.from_numpy(cur), key, shp, depth)
        out["mask." + key] = np.asarray(mk)
        out["shape." + key] = np.asarray(shp, dtype=np.int64)
    return out


def overlap_case():
    b, poses, cur = scenes.room0_window()
    cam = SimpleNamespace(**scenes.ROOM0_CAM)
    mp = object.__new__(ref_mapper_mod.Mapper)
    mp.__dict__.update(H=cam.H, W=cam.W, fx=cam.fx, fy=cam.fy, cx=cam.cx, cy=cam.cy, device="cpu",
                       bound=torch.from_numpy(b))
    depth = torch.from_numpy(scenes.box_depth(cur, scenes.ROOM0_CAM, b, seed=301))
    color = torch.from_numpy(scenes.color_image(scenes.ROOM0_CAM, seed=302))
    kf = [{"est_c2w": torch.from_numpy(p)} for p in poses]
    scores = []

    def sorted_rec(lst, **k):
        scores.extend((d["id"], float(d["percent_inside"])) for d in lst)
        return sorted(lst, **k)

    ref_mapper_mod.sorted = sorted_rec
    np.random.seed(11)
    try:
        with fixed_draws(25):
            sel = mp.keyframe_selection_overlap(color, depth, torch.from_numpy(cur), kf, 3)
    finally:
        del ref_mapper_mod.sorted
    return {"depth_seed": np.int64(301), "color_seed": np.int64(302), "draw_seed": np.int64(25),
            "np_seed": np.int64(11), "scores": np.asarray([s for _, s in sorted(scores)]),
            "selected": np.asarray(sel, dtype=np.int64), "k": np.int64(3)}


def np_dict(prefix, d):
    return {prefix + k: (v.detach().numpy() if torch.is_tensor(v) else np.asarray(v)) for k, v in d.items()}


def main():
    gen = torch.Generator().manual_seed(4321)
    out = {}
    out.update(np_dict("camera.", camera_case(gen)))
    out.update(np_dict("tloss_hd.", tracker_loss_case(gen, True)))
    out.update(np_dict("tloss_nohd.", tracker_loss_case(gen, False)))
    out.update(np_dict("mloss_color.", mapper_loss_case(gen, "color")))
    out.update(np_dict("mloss_middle.", mapper_loss_case(gen, "middle")))
    out.update(np_dict("track.", tracker_loop_case()))
    out.update(np_dict("map.", mapper_loop_case()))
    out.update(np_dict("frustum.", frustum_case()))
    out.update(np_dict("overlap.", overlap_case()))
    path = os.path.join(HERE, "loop_fixtures.npz")
    np.savez_compressed(path, **{k: (np.ascontiguousarray(v) if np.ndim(v) else np.asarray(v)) for k, v in out.items()})
    print("wrote", path, os.path.getsize(path) // 1024, "KiB", len(out), "arrays")
    print("map losses", out["map.losses"], "selected", out["map.selected"])
    print("track losses", out["track.losses"])
    print("overlap scores", out["overlap.scores"], "selected", out["overlap.selected"])
    for k in ("grid_middle", "grid_fine", "grid_color"):
        print("frustum", k, out["frustum.mask." + k].shape, int(out["frustum.mask." + k].sum()))


if __name__ == "__main__":
    main()
