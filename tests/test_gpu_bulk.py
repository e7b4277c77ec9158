"""Forward-only bulk queries on the HIP kernels vs the oracle:

  Renderer.render_img  (Renderer.py:200-255): full-image render in ray batches, each batch with
                        its own batch-global max(gt_depth) (render_batch_ray per batch, no inside mask)
  Renderer.eval_points (Renderer.py:23-61) over a large point set, as Mesher.eval_points /
                        get_mesh call it (Mesher.py:281-319,382-433) — fine (occupancy) and colour

Tolerance: SURVEY §8(c) forward bar — max-abs ≤ 2e-4 and rel-L2 ≤ 1e-4.
"""
import importlib

import pytest
import torch

from conftest import grids_from, rel_l2, sd_from
from oracle import nslam_oracle as orc
from test_gpu_dropins import Scene, base_cfg

pytestmark = pytest.mark.gpu
P = importlib.import_module("nice-slam_amd")
DEV = torch.device("cuda:0")


@pytest.mark.parametrize("with_gt", [True, False])
def test_render_img_matches_oracle(tiny, with_gt):
    H, W, bs = 24, 32, 300                     # 768 rays in batches of 300, 300, 168
    sc = Scene(tiny, H, W)
    cfg = base_cfg()
    s = sc.slam(cfg)
    r = P.Renderer(cfg, None, s, ray_batch_size=bs)
    gt = sc.depth.to(DEV) if with_gt else None
    with torch.no_grad():
        depth, unc, color = r.render_img(s.shared_c, s.shared_decoders, sc.c2w.to(DEV), DEV, "color", gt_depth=gt)
    assert depth.shape == (H, W) and unc.shape == (H, W) and color.shape == (H, W, 3)
    assert depth.dtype == torch.float64 and unc.dtype == torch.float64
    jj, ii = torch.meshgrid(torch.arange(H, dtype=torch.float32), torch.arange(W, dtype=torch.float32), indexing="ij")
    ro, rd = orc.rays_from_uv(ii.reshape(-1), jj.reshape(-1), sc.c2w, sc.fx, sc.fy, sc.cx, sc.cy)
    sd = {k: v for k, v in sc.sd.items() if not k.startswith("coarse")}
    ds, us, cs = [], [], []
    for i in range(0, H * W, bs):
        g = sc.depth.reshape(-1)[i:i + bs] if with_gt else None
        d, u, c = orc.render_batch_ray(sd, sc.grids, rd[i:i + bs], ro[i:i + bs], "color", sc.bound, g)
        ds.append(d)
        us.append(u)
        cs.append(c)
    d_ref, u_ref, c_ref = torch.cat(ds).reshape(H, W), torch.cat(us).reshape(H, W), torch.cat(cs).reshape(H, W, 3)
    for got, ref in ((depth, d_ref), (unc, u_ref), (color, c_ref)):
        got = got.cpu().to(ref.dtype)
        assert float((got - ref).abs().max()) <= 2e-4
        assert rel_l2(got, ref) <= 1e-4


@pytest.mark.parametrize("stage", ["fine", "color"])
def test_bulk_eval_points_matches_oracle(tiny, stage):
    """200k points (several fused-query launches' worth of tiles, incl. out-of-bound points that
    get the occupancy logit 100) under no_grad, as the mesher queries them."""
    sc = Scene(tiny)
    s = sc.slam(base_cfg())
    g = torch.Generator().manual_seed(4)
    lo, hi = sc.bound[:, 0], sc.bound[:, 1]
    p = (lo + (hi - lo) * (torch.rand(200_000, 3, generator=g, dtype=torch.float64) * 1.1 - 0.05))
    with torch.no_grad():
        raw = s.renderer.eval_points(p.to(DEV), s.shared_decoders, s.shared_c, stage, DEV)
    sd = {k: v for k, v in sc.sd.items() if not k.startswith("coarse")}
    ref = orc.eval_points(sd, p, sc.grids, stage, sc.bound)
    got = raw.cpu()
    assert float((got - ref).abs().max()) <= 2e-4
    assert rel_l2(got, ref) <= 1e-4
    assert bool((got[:, 3] == 100).any())  # some points are outside the bound
