"""Generate golden vectors from the REFERENCE's own hot-path modules (build container only).

Run:  PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports ``src.common``, ``src.conv_onet.models.decoder`` and ``src.utils.Renderer`` from the
read-only reference checkout, feeds them seeded inputs and writes inputs + outputs + VJPs (fixed
random cotangents) as numpy ``.npz`` files next to this script.  Nothing here runs on the GPU box;
the committed ``.npz`` files are the data the tests use there.

Harness notes:
  * ``NICE.forward`` builds ``cuda:{p.get_device()}`` (decoder.py:316), so on CPU only stage
    'color' runs through it; the other stages go through ``StageCombiner``, which calls the
    reference sub-decoders and applies the 4-line combiner of decoder.py:317-335.
  * Decoder parameters come from ``oracle.init_decoders`` (seeded) and are loaded into the
    reference ``NICE`` module with ``load_state_dict`` so both sides see identical weights.
"""
import os
import sys
from types import SimpleNamespace

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import nslam_oracle as orc  # noqa: E402

from src.common import get_rays_from_uv, raw2outputs_nerf_color  # noqa: E402  (reference)
from src.conv_onet.models.decoder import NICE  # noqa: E402  (reference)
from src.utils.Renderer import Renderer  # noqa: E402  (reference)

torch.set_num_threads(8)

# tiny non-cubic scene so axis-order bugs show up; grid_len values are config data
TINY_BOUND = [[0.0, 3.0], [-0.5, 2.2], [0.2, 2.5]]
TINY_LEN = {"coarse": 2.0, "middle": 0.64, "fine": 0.32, "color": 0.32, "bound_divisible": 0.32}


class StageCombiner:
    """Harness: stage combiner of decoder.py:317-335 over the reference sub-decoders (CPU-safe)."""

    def __init__(self, nice):
        self.m = nice

    def __call__(self, p, c_grid, stage="middle"):
        m = self.m
        if stage == "color":
            return m(p, c_grid, stage)
        if stage == "coarse":
            occ = m.coarse_decoder(p, c_grid).squeeze(0)
        elif stage == "middle":
            occ = m.middle_decoder(p, c_grid).squeeze(0)
        else:
            occ = m.fine_decoder(p, c_grid) + m.middle_decoder(p, c_grid).squeeze(0)
        raw = torch.zeros(occ.shape[0], 4)
        raw[..., -1] = occ
        return raw


def ref_nice(sd, bound):
    m = NICE(dim=3, c_dim=32, coarse_grid_len=TINY_LEN["coarse"], middle_grid_len=TINY_LEN["middle"],
             fine_grid_len=TINY_LEN["fine"], color_grid_len=TINY_LEN["color"], hidden_size=32,
             coarse=True, pos_embedding_method="fourier")
    m.load_state_dict({k: v.clone() for k, v in sd.items()})
    for d in (m.middle_decoder, m.fine_decoder, m.color_decoder):
        d.bound = bound
    m.coarse_decoder.bound = bound * 2
    return m


def ref_renderer(bound, n_strat=32, n_surf=16):
    cfg = {"rendering": {"N_samples": n_strat, "N_surface": n_surf, "N_importance": 0,
                         "lindisp": False, "perturb": 0.0}, "scale": 1, "occupancy": True}
    slam = SimpleNamespace(nice=True, bound=bound, H=680, W=1200, fx=600.0, fy=600.0, cx=599.5, cy=339.5)
    return Renderer(cfg, None, slam)


def make_rays(bound, n, gen, zero_frac=0.125):
    """Camera-like rays from near the bound centre, gt depth = fraction of the AABB exit distance."""
    ctr = bound.mean(1).float()
    ang = torch.rand(3, generator=gen) * 2 * np.pi
    c, s = torch.cos(ang), torch.sin(ang)
    rz = torch.tensor([[c[0], -s[0], 0], [s[0], c[0], 0], [0, 0, 1]])
    rx = torch.tensor([[1, 0, 0], [0, c[1], -s[1]], [0, s[1], c[1]]])
    R = (rz @ rx).float()
    i = torch.rand(n, generator=gen) * 1200
    j = torch.rand(n, generator=gen) * 680
    c2w = torch.eye(4)
    c2w[:3, :3] = R
    c2w[:3, 3] = ctr + (torch.rand(3, generator=gen) - 0.5) * 0.2
    rays_o, rays_d = get_rays_from_uv(i, j, c2w, 680, 1200, 600.0, 600.0, 599.5, 339.5, "cpu")
    far = orc.far_bound(rays_o, rays_d, bound).float()
    gt = far * (0.5 + 0.45 * torch.rand(n, generator=gen))
    gt[torch.randperm(n, generator=gen)[: int(n * zero_frac)]] = 0.0
    return i, j, c2w, rays_o.float().contiguous(), rays_d.float().contiguous(), gt.float()


def np_dict(prefix, d):
    return {prefix + k: (v.detach().numpy() if torch.is_tensor(v) else np.asarray(v)) for k, v in d.items()}


def render_case(sd, grids, bound, rays_o, rays_d, gt, stage, gen, n_strat=32, n_surf=16):
    m = ref_nice(sd, bound)
    comb = StageCombiner(m)
    r = ref_renderer(bound, n_strat, n_surf)
    gr = {k: v.clone().requires_grad_(True) for k, v in grids.items()}
    ro = rays_o.clone().requires_grad_(True)
    rd = rays_d.clone().requires_grad_(True)
    depth, var, color = r.render_batch_ray(gr, comb, rd, ro, "cpu", stage,
                                           gt_depth=None if gt is None else gt.clone())
    gd = torch.randn(depth.shape, generator=gen, dtype=torch.float64)
    gv = torch.randn(var.shape, generator=gen, dtype=torch.float64)
    gc = torch.randn(color.shape, generator=gen, dtype=torch.float32)
    params = dict(m.named_parameters())
    names = list(gr) + ["rays_o", "rays_d"] + list(params)
    tens = list(gr.values()) + [ro, rd] + list(params.values())
    grads = torch.autograd.grad((depth, var, color), tens, (gd, gv, gc), allow_unused=True)
    out = {"depth": depth, "var": var, "color": color, "cot_depth": gd, "cot_var": gv, "cot_color": gc}
    for n, g in zip(names, grads):
        if g is not None:
            out["grad." + n] = g
    return out


def eval_points_case(sd, grids, bound, stage, gen, M=300):
    m = ref_nice(sd, bound)
    r = ref_renderer(bound)
    lo, hi = bound[:, 0], bound[:, 1]
    p = lo + (hi - lo) * (torch.rand(M, 3, generator=gen, dtype=torch.float64) * 1.2 - 0.1)
    p[:8] = lo + (hi - lo) * torch.rand(8, 3, generator=gen, dtype=torch.float64)
    p[0, 0] = lo[0]  # exactly on the boundary: OOB under the strict test
    p[1, 1] = hi[1]
    p[2] = lo.clone()
    p[3] = hi.clone()
    gr = {k: v.clone().requires_grad_(True) for k, v in grids.items()}
    pp = p.clone().requires_grad_(True)
    raw = r.eval_points(pp, StageCombiner(m), gr, stage, "cpu")
    cot = torch.randn(raw.shape, generator=gen)
    params = dict(m.named_parameters())
    names = ["pts"] + list(gr) + list(params)
    tens = [pp] + list(gr.values()) + list(params.values())
    grads = torch.autograd.grad(raw, tens, cot, allow_unused=True)
    out = {"pts": p, "raw": raw, "cot_raw": cot}
    for n, g in zip(names, grads):
        if g is not None:
            out["grad." + n] = g
    return out


def composite_case(gen, N=96, S=48):
    raw = torch.randn(N, S, 4, generator=gen) * 0.3
    raw[:, :, 3] = torch.randn(N, S, generator=gen) * 0.4
    raw[::7, 20:, 3] = 100.0  # OOB samples: alpha == 1 exactly
    raw[::5, 10:14, 3] = 3.0
    z = torch.sort(torch.rand(N, S, generator=gen, dtype=torch.float64) * 6, -1).values
    rays_d = torch.randn(N, 3, generator=gen)
    rr = raw.clone().requires_grad_(True)
    # the reference writes raw[...,3] in place (common.py:233): feed it a non-leaf
    depth, var, rgb, w = raw2outputs_nerf_color(rr * 1.0, z, rays_d, occupancy=True, device="cpu")
    gd = torch.randn(N, generator=gen, dtype=torch.float64)
    gv = torch.randn(N, generator=gen, dtype=torch.float64)
    gc = torch.randn(N, 3, generator=gen)
    (g,) = torch.autograd.grad((depth, var, rgb), (rr,), (gd, gv, gc))
    return {"raw": raw, "z": z, "depth": depth, "var": var, "rgb": rgb, "weights": w.detach(),
            "cot_depth": gd, "cot_var": gv, "cot_color": gc, "grad.raw": g}


def main():
    gen = torch.Generator().manual_seed(1234)
    bound = orc.enlarge_bound(TINY_BOUND, TINY_LEN["bound_divisible"])
    grids = orc.make_grids(bound, TINY_LEN, gen=gen)
    # give the fine grid the same scale as the others so its gradients are not negligible in tests
    grids["grid_fine"] = grids["grid_fine"] * 100
    sd = orc.init_decoders(gen)
    i, j, c2w, rays_o, rays_d, gt = make_rays(bound, 64, gen)

    out = {"bound": bound, "ray_i": i, "ray_j": j, "c2w": c2w, "rays_o": rays_o, "rays_d": rays_d,
           "gt_depth": gt}
    out.update(np_dict("", grids))
    out.update(np_dict("sd.", sd))
    # rays_from_uv parity (common.py:74-89)
    ro2, rd2 = get_rays_from_uv(i, j, c2w, 680, 1200, 600.0, 600.0, 599.5, 339.5, "cpu")
    out["uv.rays_o"], out["uv.rays_d"] = ro2.numpy(), rd2.numpy()
    for stage in orc.STAGES:
        res = render_case(sd, grids, bound, rays_o, rays_d, gt, stage, gen)
        out.update(np_dict(f"render.{stage}.", res))
    res = render_case(sd, grids, bound, rays_o, rays_d, None, "color", gen)
    out.update(np_dict("render.color_nogt.", res))
    for stage in orc.STAGES:
        out.update(np_dict(f"eval.{stage}.", eval_points_case(sd, grids, bound, stage, gen)))
    out.update(np_dict("composite.", composite_case(gen)))
    path = os.path.join(HERE, "tiny_scene.npz")
    np.savez_compressed(path, **{k: np.ascontiguousarray(v) for k, v in out.items()})
    print("wrote", path, os.path.getsize(path) // 1024, "KiB", len(out), "arrays")

    # room0-shape case: inputs regenerated from seeds by the oracle; outputs + grad norms stored
    room = room0_case()
    path = os.path.join(HERE, "room0_color.npz")
    np.savez_compressed(path, **room)
    print("wrote", path, os.path.getsize(path) // 1024, "KiB")


ROOM0_BOUND = [[-2.9, 8.9], [-3.2, 5.5], [-3.5, 3.3]]       # configs/Replica/room0.yaml:3
ROOM0_LEN = {"coarse": 2.0, "middle": 0.32, "fine": 0.16, "color": 0.16, "bound_divisible": 0.32}


def room0_inputs(n_rays=1000, seed=7):
    """Deterministic room0-shape inputs (CPU torch RNG); shared with the tests via the oracle."""
    gen = torch.Generator().manual_seed(seed)
    bound = orc.enlarge_bound(ROOM0_BOUND, ROOM0_LEN["bound_divisible"])
    grids = orc.make_grids(bound, ROOM0_LEN, gen=gen)
    sd = orc.init_decoders(gen)
    i, j, c2w, rays_o, rays_d, gt = make_rays(bound, n_rays, gen, zero_frac=0.05)
    return bound, grids, sd, rays_o, rays_d, gt


def room0_case():
    gen = torch.Generator().manual_seed(99)
    bound, grids, sd, rays_o, rays_d, gt = room0_inputs()
    res = render_case(sd, grids, bound, rays_o, rays_d, gt, "color", gen)
    out = {"bound": bound.numpy(), "rays_o": rays_o.numpy(), "rays_d": rays_d.numpy(), "gt_depth": gt.numpy()}
    for k in ("depth", "var", "color", "cot_depth", "cot_var", "cot_color", "grad.rays_o", "grad.rays_d"):
        out[k] = res[k].detach().numpy()
    for k, v in res.items():
        if k.startswith("grad."):
            out["norm." + k] = np.float64(v.double().norm().item())
            out["sum." + k] = np.float64(v.double().sum().item())
    for k, v in grids.items():
        out["checksum." + k] = np.float64(v.double().sum().item())
    return out


if __name__ == "__main__":
    main()
