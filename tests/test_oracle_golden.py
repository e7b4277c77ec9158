"""Pin the oracle (oracle/nslam_oracle.py) against golden vectors made by the reference itself.

The golden vectors come from importing the reference's hot-path modules in the build container
(tests/golden/make_golden.py).  The oracle uses the same torch CPU kernels, so agreement is
expected to be (nearly) bitwise; tolerances below are at the fp64/fp32 rounding floor.
"""
import numpy as np
import pytest
import torch

from conftest import grids_from, rel_l2, sd_from
from oracle import nslam_oracle as orc

STAGES = list(orc.STAGES) + ["color_nogt"]


def _render(tiny, stage):
    sd = {k: v.clone().requires_grad_(True) for k, v in sd_from(tiny).items()}
    grids = {k: v.clone().requires_grad_(True) for k, v in grids_from(tiny).items()}
    ro = torch.from_numpy(tiny["rays_o"]).requires_grad_(True)
    rd = torch.from_numpy(tiny["rays_d"]).requires_grad_(True)
    bound = torch.from_numpy(tiny["bound"])
    gt = None if stage == "color_nogt" else torch.from_numpy(tiny["gt_depth"])
    st = "color" if stage == "color_nogt" else stage
    depth, var, color = orc.render_batch_ray(sd, grids, rd, ro, st, bound, gt)
    pre = f"render.{stage}."
    cots = tuple(torch.from_numpy(tiny[pre + k]) for k in ("cot_depth", "cot_var", "cot_color"))
    names = list(grids) + ["rays_o", "rays_d"] + list(sd)
    tens = list(grids.values()) + [ro, rd] + list(sd.values())
    grads = torch.autograd.grad((depth, var, color), tens, cots, allow_unused=True)
    return pre, depth, var, color, dict(zip(names, grads))


@pytest.mark.parametrize("stage", STAGES)
def test_render_batch_ray_matches_reference(tiny, stage):
    pre, depth, var, color, grads = _render(tiny, stage)
    np.testing.assert_allclose(depth.detach().numpy(), tiny[pre + "depth"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(var.detach().numpy(), tiny[pre + "var"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(color.detach().numpy(), tiny[pre + "color"], rtol=0, atol=1e-6)
    golden = {k[len(pre) + 5:]: v for k, v in tiny.items() if k.startswith(pre + "grad.")}
    for name, g in grads.items():
        if name not in golden:
            assert g is None or float(g.abs().max()) == 0.0, name
            continue
        assert g is not None, name
        assert rel_l2(g.numpy(), golden[name]) < 1e-5, name


@pytest.mark.parametrize("stage", orc.STAGES)
def test_eval_points_matches_reference(tiny, stage):
    sd = {k: v.clone().requires_grad_(True) for k, v in sd_from(tiny).items()}
    grids = {k: v.clone().requires_grad_(True) for k, v in grids_from(tiny).items()}
    pre = f"eval.{stage}."
    p = torch.from_numpy(tiny[pre + "pts"]).clone().requires_grad_(True)
    bound = torch.from_numpy(tiny["bound"])
    raw = orc.eval_points(sd, p, grids, stage, bound)
    np.testing.assert_allclose(raw.detach().numpy(), tiny[pre + "raw"], rtol=0, atol=1e-6)
    names = ["pts"] + list(grids) + list(sd)
    tens = [p] + list(grids.values()) + list(sd.values())
    grads = torch.autograd.grad(raw, tens, torch.from_numpy(tiny[pre + "cot_raw"]), allow_unused=True)
    for name, g in zip(names, grads):
        key = pre + "grad." + name
        if key not in tiny:
            assert g is None or float(g.abs().max()) == 0.0, name
            continue
        assert rel_l2(g.numpy(), tiny[key]) < 1e-5, name


def test_composite_matches_reference(tiny):
    raw = torch.from_numpy(tiny["composite.raw"]).requires_grad_(True)
    z = torch.from_numpy(tiny["composite.z"])
    depth, var, rgb, w = orc.composite(raw, z)
    np.testing.assert_array_equal(depth.detach().numpy(), tiny["composite.depth"])
    np.testing.assert_array_equal(var.detach().numpy(), tiny["composite.var"])
    np.testing.assert_array_equal(rgb.detach().numpy(), tiny["composite.rgb"])
    cots = tuple(torch.from_numpy(tiny["composite." + k]) for k in ("cot_depth", "cot_var", "cot_color"))
    (g,) = torch.autograd.grad((depth, var, rgb), (raw,), cots)
    np.testing.assert_allclose(g.numpy(), tiny["composite.grad.raw"], rtol=1e-6, atol=1e-7)


def test_rays_from_uv_matches_reference(tiny):
    i, j = torch.from_numpy(tiny["ray_i"]), torch.from_numpy(tiny["ray_j"])
    ro, rd = orc.rays_from_uv(i, j, torch.from_numpy(tiny["c2w"]), 600.0, 600.0, 599.5, 339.5)
    np.testing.assert_array_equal(ro.numpy(), tiny["uv.rays_o"])
    np.testing.assert_array_equal(rd.numpy(), tiny["uv.rays_d"])


def test_room0_oracle_reproduces_golden(room0):
    """room0-shape inputs are regenerated from seeds (grids, decoders) + stored rays."""
    gen = torch.Generator().manual_seed(7)
    bound = orc.enlarge_bound([[-2.9, 8.9], [-3.2, 5.5], [-3.5, 3.3]], 0.32)
    np.testing.assert_array_equal(bound.numpy(), room0["bound"])
    grids = orc.make_grids(bound, {"coarse": 2.0, "middle": 0.32, "fine": 0.16, "color": 0.16}, gen=gen)
    for k, v in grids.items():
        assert float(v.double().sum()) == pytest.approx(float(room0["checksum." + k]), rel=0, abs=1e-9)
    sd = orc.init_decoders(gen)
    ro = torch.from_numpy(room0["rays_o"])
    rd = torch.from_numpy(room0["rays_d"])
    gt = torch.from_numpy(room0["gt_depth"])
    depth, var, color = orc.render_batch_ray(sd, grids, rd, ro, "color", bound, gt)
    np.testing.assert_allclose(depth.numpy(), room0["depth"], rtol=0, atol=1e-10)
    np.testing.assert_allclose(color.numpy(), room0["color"], rtol=0, atol=1e-6)
