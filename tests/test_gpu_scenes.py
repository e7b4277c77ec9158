"""GPU parity at the grid shapes of the other BASELINE.json configs.

The golden vectors pin the oracle on a tiny scene and on room0; these cases run the HIP path and
the oracle on the same seeded inputs at the real grid shapes of Demo (configs/Demo/demo.yaml:28),
ScanNet scene0000 (configs/ScanNet/scene0000.yaml:3) and Apartment
(configs/Apartment/apartment.yaml:24, full coarse → fine hierarchy), so non-cubic extents,
int()-truncated axes (Apartment fine x = 107, Demo middle x = 20) and the coarse grid's ×2 bound
(NICE_SLAM.py:152-157) are indexed correctly.  192 rays keep the CPU oracle to seconds.

The 512³×32 stress grid (BASELINE configs[4], 16 GiB) is too large for the CPU oracle: it is
checked against torch's F.grid_sample on the device (the semantics decoder.py:168-175 calls:
bilinear, border, align_corners=True) at 2^20 points, plus a size-independent property of the
scatter (every trilinear weight set sums to 1).

Tolerances as tests/test_gpu_parity.py (the reference's own fp32 noise floor).
"""
import json
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import load_pkg, rel_l2
from oracle import nslam_oracle as orc

pytestmark = pytest.mark.gpu

FWD_ABS, FWD_REL = 2e-4, 1e-4
LENS = {"coarse": 2.0, "middle": 0.32, "fine": 0.16, "color": 0.16}  # configs/nice_slam.yaml:7-12
SCENES = {  # bound from the scene yaml; shapes from SURVEY.md §8 ([1, C, Z, Y, X])
    "demo": ([[0.0, 6.5], [0.0, 4.0], [0.0, 3.5]], ("coarse", "middle", "fine", "color"),
             {"grid_coarse": [1, 32, 3, 4, 6], "grid_middle": [1, 32, 10, 12, 20],
              "grid_fine": [1, 32, 21, 25, 41]}),
    "scene0000": ([[-2.0, 11.0], [-2.0, 11.5], [-2.0, 5.5]], ("middle", "fine", "color"),
                  {"grid_middle": [1, 32, 23, 42, 40], "grid_fine": [1, 32, 47, 85, 81]}),
    "apartment": ([[-5.8, 11.3], [-4.0, 4.5], [-7.9, 4.9]], ("coarse", "middle", "fine", "color"),
                  {"grid_coarse": [1, 32, 13, 8, 17], "grid_middle": [1, 32, 40, 26, 53],
                   "grid_fine": [1, 32, 81, 53, 107], "grid_color": [1, 32, 81, 53, 107]}),
}


def tol_for(name):
    if name.startswith("grid_middle") or name in ("rays_o", "rays_d"):
        return 5e-3
    if name.startswith("grid_fine"):
        return 1e-3
    return 2e-4


def scene_inputs(name, n_rays, seed):
    bound_cfg, _, shapes = SCENES[name]
    bound = orc.enlarge_bound(bound_cfg, 0.32)
    gen = torch.Generator().manual_seed(seed)
    grids = orc.make_grids(bound, LENS, gen=gen)
    for k, shp in shapes.items():
        assert list(grids[k].shape) == shp, (k, grids[k].shape)
    sd = orc.init_decoders(gen)
    # rays from near the bound centre in random directions; depth inside the box; 5 % zero depths
    # (the gt==0 surface branch, Renderer.py:140-150)
    lo, hi = bound[:, 0].float(), bound[:, 1].float()
    ro = (lo + hi) / 2 + (torch.rand(n_rays, 3, generator=gen) - 0.5) * (hi - lo) * 0.3
    rd = torch.randn(n_rays, 3, generator=gen)
    rd = rd / rd.norm(dim=1, keepdim=True)
    far = orc.far_bound(ro, rd, bound).float()
    gt = far * (0.5 + 0.45 * torch.rand(n_rays, generator=gen))
    gt[torch.rand(n_rays, generator=gen) < 0.05] = 0
    return bound, grids, sd, ro.contiguous(), rd.contiguous(), gt


@pytest.mark.parametrize("name,stage", [(n, s) for n in SCENES for s in SCENES[n][1]])
def test_scene_render_matches_oracle(name, stage):
    pkg = load_pkg()
    dev = torch.device("cuda:0")
    bound, grids, sd, ro, rd, gt = scene_inputs(name, 192, seed=31 + len(name))
    nice = pkg.NICE(dim=3, c_dim=32, coarse_grid_len=2.0, middle_grid_len=0.32, fine_grid_len=0.16,
                    color_grid_len=0.16, hidden_size=32, coarse=True)
    nice.load_state_dict({k: v.clone() for k, v in sd.items()})
    nice.set_bound(bound)
    nice = nice.to(dev)
    cfg = {"rendering": {"N_samples": 32, "N_surface": 16, "N_importance": 0, "lindisp": False, "perturb": 0.0},
           "scale": 1, "occupancy": True}
    r = pkg.Renderer(cfg, None, SimpleNamespace(nice=True, bound=bound, H=480, W=640, fx=577.6, fy=578.7,
                                                cx=318.9, cy=242.7))
    gd = {k: v.to(dev).contiguous(memory_format=torch.channels_last_3d).requires_grad_(True)
          for k, v in grids.items()}
    rod, rdd = ro.to(dev).requires_grad_(True), rd.to(dev).requires_grad_(True)
    depth, var, color = r.render_batch_ray(gd, nice, rdd, rod, dev, stage, gt_depth=gt.to(dev))

    gc = {k: v.clone().requires_grad_(True) for k, v in grids.items()}
    roc, rdc = ro.clone().requires_grad_(True), rd.clone().requires_grad_(True)
    sdc = {k: v.clone().requires_grad_(k.startswith("color_decoder.")) for k, v in sd.items()}
    d_ref, v_ref, c_ref = orc.render_batch_ray(sdc, gc, rdc, roc, stage, bound, gt)

    report, ok = {}, True
    for nm, a, b in (("depth", depth, d_ref), ("var", var, v_ref), ("color", color, c_ref)):
        a_, b_ = a.detach().cpu().double().numpy(), b.detach().double().numpy()
        e = {"max_abs": float(np.abs(a_ - b_).max()), "rel_l2": rel_l2(a_, b_)}
        report[nm] = e
        ok &= e["max_abs"] <= FWD_ABS and e["rel_l2"] <= FWD_REL
    g = torch.Generator().manual_seed(5)
    cots = (torch.randn(d_ref.shape, generator=g, dtype=d_ref.dtype),
            torch.randn(v_ref.shape, generator=g, dtype=v_ref.dtype) * 0.1,
            torch.randn(c_ref.shape, generator=g, dtype=c_ref.dtype))
    dec = [k for k in sdc if k.startswith("color_decoder.")] if stage == "color" else []
    names = list(gc) + ["rays_o", "rays_d"] + dec
    ref_g = torch.autograd.grad((d_ref, v_ref, c_ref), [gc[k] for k in gc] + [roc, rdc] + [sdc[k] for k in dec],
                                cots, allow_unused=True)
    params = dict(nice.named_parameters())
    got_g = torch.autograd.grad((depth, var, color), [gd[k] for k in gc] + [rod, rdd] + [params[k] for k in dec],
                                tuple(c.to(dev) for c in cots), allow_unused=True)
    for nm, a, b in zip(names, got_g, ref_g):
        if b is None or float(b.abs().max()) == 0.0:
            ok &= a is None or float(a.abs().max()) == 0.0
            continue
        report[nm] = rel_l2(a, b)
        ok &= report[nm] <= tol_for(nm)
    assert ok, json.dumps(report, indent=1)


def test_stress_grid_query_matches_torch():
    """BASELINE configs[4]: the standalone grid query on a 512³×32 channels-last grid (16 GiB)."""
    pkg = load_pkg()
    dev = torch.device("cuda:0")
    n = 512
    grid = torch.empty(1, n, n, n, 32, device=dev).permute(0, 4, 1, 2, 3)  # [1,32,Z,Y,X], channels-last
    assert grid.is_contiguous(memory_format=torch.channels_last_3d)
    grid.normal_(0, 0.01, generator=torch.Generator(device=dev).manual_seed(0))
    coords = torch.rand(1 << 20, 3, device=dev, generator=torch.Generator(device=dev).manual_seed(1)) * 2.2 - 1.1
    coords[:6] = torch.tensor([[-1, -1, -1], [1, 1, 1], [1, -1, 0.3], [0, 0, 0], [-1.05, 0.5, 1], [1.0, 1.0, -1.0]],
                              device=dev)
    out = pkg.ops.grid_sample(grid, coords)
    ref = F.grid_sample(grid, coords.reshape(1, -1, 1, 1, 3), mode="bilinear", padding_mode="border",
                        align_corners=True).reshape(32, -1).t()
    assert float((out - ref).abs().max()) < 1e-6
    del out, ref
    # backward: scatter ones for 2^18 points into the 16 GiB gradient.  Size-independent property:
    # the total is (#points × 32) since each trilinear weight set sums to 1.  Spot check: z rows
    # 0..5 against torch's grid gradient over an 8-deep slab (points with z index < 6.5 are the
    # only ones touching rows 0..5; the slab's z-extent maps index k to k)
    m = 1 << 18
    c2 = coords[:m].contiguous()
    g0 = grid.detach().requires_grad_(True)
    o2 = pkg.ops.grid_sample(g0, c2)
    (gg,) = torch.autograd.grad(o2, (g0,), torch.ones_like(o2))
    del grid, g0, o2
    total = float(gg.sum(dtype=torch.float64))
    assert abs(total - m * 32) / (m * 32) < 1e-6, total
    zi = ((c2[:, 2] + 1) / 2 * (n - 1)).clamp(0, n - 1)
    cs = c2[zi < 6.5]
    zf = ((cs[:, 2] + 1) / 2 * (n - 1)).clamp(min=0) / 7 * 2 - 1
    gref = torch.zeros(1, 32, 8, n, n, device=dev, requires_grad=True)
    oref = F.grid_sample(gref, torch.stack([cs[:, 0], cs[:, 1], zf], 1).reshape(1, -1, 1, 1, 3), mode="bilinear",
                         padding_mode="border", align_corners=True)
    (gr,) = torch.autograd.grad(oref, (gref,), torch.ones_like(oref))
    assert rel_l2(gg[:, :, :6], gr[:, :, :6]) < 1e-5
