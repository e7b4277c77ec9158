"""Direct sub-decoder calls (MLP.forward / MLP_no_xyz.forward, decoder.py:177-203, 262-274) through
the fused kernel vs the oracle's restatement of the same modules on the device: the reference's
NICE.forward calls them one by one (decoder.py:312-342), so code that does the same must work on the
drop-in.  Forward max-abs 2e-4; gradients (own grid, the decoder's parameters, the points) at the
VJP tolerances of tests/test_gpu_parity.py."""
import pytest
import torch

from conftest import grids_from, rel_l2, sd_from
from oracle import nslam_oracle as orc

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
TOL = {"coarse": 2e-4, "middle": 5e-3, "fine": 1e-3, "color": 2e-4}


def oracle_decoder(sd, name, p, grids, bound):
    if name == "coarse":
        return orc.mlp_no_xyz(sd, "coarse_decoder.", orc.grid_features(p, grids["grid_coarse"], bound * 2))[:, 0]
    if name == "middle":
        return orc.mlp_xyz(sd, "middle_decoder.", p, orc.grid_features(p, grids["grid_middle"], bound))[:, 0]
    if name == "fine":
        f = torch.cat([orc.grid_features(p, grids["grid_fine"], bound),
                       orc.grid_features(p, grids["grid_middle"], bound).detach()], 1)
        return orc.mlp_xyz(sd, "fine_decoder.", p, f)[:, 0]
    return orc.mlp_xyz(sd, "color_decoder.", p, orc.grid_features(p, grids["grid_color"], bound))


@pytest.mark.parametrize("name", ["coarse", "middle", "fine", "color"])
def test_sub_decoder_direct_call(pkg, tiny, name):
    bound = torch.from_numpy(tiny["bound"])
    sd = sd_from(tiny)
    nice = pkg.NICE(c_dim=32, coarse_grid_len=2.0, middle_grid_len=0.64, fine_grid_len=0.32, color_grid_len=0.32,
                    hidden_size=32, coarse=True)
    nice.load_state_dict(sd)
    nice.set_bound(bound)
    nice = nice.to(DEV)
    g = torch.Generator().manual_seed(5)
    n = 1500
    p = (bound[:, 0] + torch.rand(n, 3, generator=g, dtype=torch.float64) * (bound[:, 1] - bound[:, 0])).to(DEV)
    grids = {k: v.to(DEV).contiguous(memory_format=torch.channels_last_3d).requires_grad_(True)
             for k, v in grids_from(tiny).items()}
    pp = p.clone().requires_grad_(True)
    dec = nice.decoder(name)
    out = dec(pp, grids)
    # oracle on the same device, reference module semantics
    sdo = {k: v.to(DEV).clone().requires_grad_(k.startswith(name + "_decoder.")) for k, v in sd.items()}
    go = {k: v.detach().clone().requires_grad_(True) for k, v in grids.items()}
    po = p.clone().requires_grad_(True)
    ref = oracle_decoder(sdo, name, po, go, bound.to(DEV))
    assert out.shape == ref.shape
    assert float((out.detach() - ref.detach()).abs().max()) < 2e-4
    w = torch.randn(ref.shape, generator=g).to(DEV)
    if name == "color":
        w[:, 3] = 0.0  # NICE.forward overwrites that row (decoder.py:341): no cotangent reaches the hidden layers
    (out * w).sum().backward()
    (ref * w).sum().backward()
    key = "grid_" + name
    assert rel_l2(grids[key].grad, go[key].grad) <= TOL[name]
    for other in set(grids) - {key}:
        assert grids[other].grad is None, other  # the fine decoder reads the middle grid under no_grad
    got = torch.cat([q.grad.reshape(-1) for q in dec.parameters()])
    exp = torch.cat([sdo[name + "_decoder." + k].grad.reshape(-1) for k, _ in dec.named_parameters()])
    assert rel_l2(got, exp) <= 2e-4
    assert rel_l2(pp.grad, po.grad) <= 5e-3


def test_color_decoder_fourth_output(pkg, tiny):
    """The colour decoder's 4th output row (h4 @ Wo[3] + bo[3], decoder.py:198-203; NICE.forward
    overwrites it, decoder.py:341, but a direct MLP(color=True) caller may differentiate it): its
    value, and a cotangent on all four rows reaching the colour grid, every decoder parameter and the
    points (ABI v17 nslam_query_cfg.g_h4), vs the oracle's module on the device."""
    bound = torch.from_numpy(tiny["bound"])
    sd = sd_from(tiny)
    nice = pkg.NICE(c_dim=32, coarse_grid_len=2.0, middle_grid_len=0.64, fine_grid_len=0.32, color_grid_len=0.32,
                    hidden_size=32, coarse=True)
    nice.load_state_dict(sd)
    nice.set_bound(bound)
    nice = nice.to(DEV)
    g = torch.Generator().manual_seed(11)
    n = 1000
    p = (bound[:, 0] + torch.rand(n, 3, generator=g, dtype=torch.float64) * (bound[:, 1] - bound[:, 0])).to(DEV)
    grids = {k: v.to(DEV).contiguous(memory_format=torch.channels_last_3d).requires_grad_(True)
             for k, v in grids_from(tiny).items()}
    sdo = {k: v.to(DEV).clone().requires_grad_(k.startswith("color_decoder.")) for k, v in sd.items()}
    go = {k: v.detach().clone().requires_grad_(True) for k, v in grids.items()}
    for rows in ((3,), (0, 1, 2, 3)):  # the 4th row alone, then all four
        for t in list(grids.values()) + list(go.values()) + list(nice.color_decoder.parameters()) + list(sdo.values()):
            t.grad = None
        pp = p.clone().requires_grad_(True)
        po = p.clone().requires_grad_(True)
        out = nice.color_decoder(pp, grids)
        ref = oracle_decoder(sdo, "color", po, go, bound.to(DEV))
        assert float((out.detach() - ref.detach()).abs().max()) < 2e-4
        w = torch.zeros(ref.shape)
        w[:, list(rows)] = torch.randn(n, len(rows), generator=g)
        w = w.to(DEV)
        (out * w).sum().backward()
        (ref * w).sum().backward()
        assert rel_l2(grids["grid_color"].grad, go["grid_color"].grad) <= TOL["color"], rows
        got = torch.cat([q.grad.reshape(-1) for q in nice.color_decoder.parameters()])
        exp = torch.cat([sdo["color_decoder." + k].grad.reshape(-1) for k, _ in nice.color_decoder.named_parameters()])
        assert rel_l2(got, exp) <= 2e-4, rows
        assert rel_l2(pp.grad, po.grad) <= 5e-3, rows
