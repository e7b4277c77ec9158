"""GPU parity of the fused mapping-iteration kernels (ABI v4) against the autograd drop-in path
and torch on the same inputs:

  nslam_gather_rays  vs common.get_samples (torch on the device, the reference's code path) and the
                        oracle's inside mask (Mapper.py:469-481)          — bit-exact
  ray-form query     vs the pts-form query (pts = o + d·z in torch)       — bit-exact
  nslam_render_loss  vs composite + the reference loss through autograd   — mapper and tracker
  nslam_adam_step    vs torch.optim.Adam(foreach=False) (dense, row-masked, per-parameter steps)
  MappingEngine      vs the autograd path (one iteration's gradients; loss decreases over 5)
"""
import ctypes
import importlib

import numpy as np
import pytest
import torch

from conftest import grids_from, rel_l2, sd_from
from oracle import nslam_oracle as orc
from test_gpu_dropins import Scene, base_cfg

pytestmark = pytest.mark.gpu
P = importlib.import_module("nice-slam_amd")
DEV = torch.device("cuda:0")


def _frames(tiny, nf=3, H=96, W=128):
    sc = Scene(tiny, H, W)
    g = torch.Generator().manual_seed(5)
    frames = []
    for f in range(nf):
        c2w = sc.c2w.clone()
        c2w[:3, 3] += (torch.rand(3, generator=g) - 0.5) * 0.2
        d = sc.depth * (0.9 + 0.2 * torch.rand(H, W, generator=g))
        d[torch.rand(H, W, generator=g) < 0.03] = 0
        frames.append((d.to(DEV), torch.rand(H, W, 3, generator=g).to(DEV), c2w.to(DEV)))
    return sc, frames


@pytest.mark.parametrize("window", [(0, 96, 0, 128), (20, 76, 20, 108)])
def test_gather_rays_bitexact(tiny, window):
    sc, frames = _frames(tiny)
    H, W = 96, 128
    h0, h1, w0, w1 = window
    n_per = 150
    pix = torch.randint((h1 - h0) * (w1 - w0), (len(frames) * n_per,), device=DEV,
                        generator=torch.Generator(device=DEV).manual_seed(1))
    ro, rd, gd, gc, keep = P.ops.gather_rays(frames, pix, n_per, H, W, window, sc.fx, sc.fy, sc.cx, sc.cy, sc.bound)
    # reference path: get_sample_uv's meshgrid + select_uv indexing + get_rays_from_uv, on the device
    for f, (d, c, m) in enumerate(frames):
        idx = pix[f * n_per:(f + 1) * n_per]
        i, j = torch.meshgrid(torch.linspace(w0, w1 - 1, w1 - w0).to(DEV), torch.linspace(h0, h1 - 1, h1 - h0).to(DEV),
                              indexing="ij")
        i, j = i.t().reshape(-1)[idx], j.t().reshape(-1)[idx]
        dd = d[h0:h1, w0:w1].reshape(-1)[idx]
        cc = c[h0:h1, w0:w1].reshape(-1, 3)[idx]
        o_ref, d_ref = P.common.get_rays_from_uv(i, j, m, H, W, sc.fx, sc.fy, sc.cx, sc.cy, DEV)
        sl = slice(f * n_per, (f + 1) * n_per)
        assert torch.equal(ro[sl], o_ref.float()), "rays_o"
        assert torch.equal(rd[sl], d_ref.float()), f"rays_d max diff {(rd[sl] - d_ref).abs().max()}"
        assert torch.equal(gc[sl], cc)
        k_ref = orc.inside_mask(o_ref.cpu(), d_ref.cpu(), dd.cpu(), sc.bound).to(DEV)
        assert torch.equal(keep[sl].bool(), k_ref)
        assert torch.equal(gd[sl], torch.where(k_ref, dd, torch.zeros_like(dd)))
    assert 0 < int(keep.sum()) < keep.numel()  # both branches of the prefilter exercised


def _nice(sc):
    s = sc.slam(base_cfg())
    return s.shared_decoders, s.shared_c


@pytest.mark.parametrize("stage", ["middle", "fine", "color"])
def test_ray_form_query_matches_pts_form(tiny, stage):
    sc, frames = _frames(tiny)
    nice, c = _nice(sc)
    eng = P.engine.MappingEngine(nice, c, sc.bound, 32, 16, device=DEV)
    pix = torch.randint(96 * 128, (3 * 64,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(2))
    ro, rd, gd, gc, keep = P.ops.gather_rays(frames, pix, 64, 96, 128, (0, 96, 0, 128), sc.fx, sc.fy, sc.cx, sc.cy)
    z = P.ops.sample_z(ro, rd, gd, sc.bound, 32, 16)
    raw = eng.query_fwd(stage, ro, rd, z)
    pts = ro[:, None, :] + rd[:, None, :] * z[:, :, None]
    raw_ref = nice(pts.reshape(-1, 3), c, stage=stage, oob_bound=sc.bound)
    assert torch.equal(raw, raw_ref)
    # backward into the engine's buffers vs autograd on the pts form
    g_raw = torch.randn_like(raw)
    trainable = ("color",) if stage == "color" else ()
    keys, dn = eng.grads_for(stage, trainable)
    eng.gbuf.zero_()
    for n in dn:
        eng.decs[n].grad.zero_()
    eng.query_bwd(stage, ro, rd, z, g_raw, keys, dn)
    gl = {k: c[k].detach().clone().requires_grad_(True) for k in c}
    for p in nice.parameters():
        p.requires_grad_(False)
    if stage == "color":
        for p in nice.color_decoder.parameters():
            p.requires_grad_(True)
    out = nice(pts.reshape(-1, 3), gl, stage=stage, oob_bound=sc.bound)
    tens = [gl[k] for k in keys] + (list(nice.color_decoder.parameters()) if stage == "color" else [])
    grads = torch.autograd.grad(out, tens, g_raw)
    for k, g in zip(keys, grads):
        assert rel_l2(eng.ggrad[k], g) < 1e-5, k
    if stage == "color":
        ref = torch.cat([g.reshape(-1) for g in grads[len(keys):]])
        assert rel_l2(eng.decs["color"].grad, ref) < 1e-5


def _autograd_loss(raw, z, gd, gc, keep, mode, use_color, handle_dynamic, w):
    raw = raw.detach().clone().requires_grad_(True)
    depth, var, color = P.ops.composite(raw.reshape(z.shape[0], z.shape[1], 4), z)
    k = keep.bool()
    d, u, col, g, c = depth[k], var[k], color[k], gd[k], gc[k]
    if mode == "mapper":  # Mapper.py:487-501
        m = g > 0
        loss = torch.abs(g[m] - d[m]).sum()
        if use_color:
            loss = loss + w * torch.abs(c - col).sum()
    else:  # Tracker.py:110-123
        u = u.detach()
        m = g > 0
        if handle_dynamic:
            tmp = torch.abs(g - d) / torch.sqrt(u + 1e-10)
            m = (tmp < 10 * tmp.median()) & (g > 0)
        loss = (torch.abs(g - d) / torch.sqrt(u + 1e-10))[m].sum()
        if use_color:
            loss = loss + w * torch.abs(c - col)[m].sum()
    loss.backward()
    return depth, var, color, loss.detach(), raw.grad


# n_per 100 (300 rays): the median by rank selection; 400 (1200 rays > 1024 threads): the bitonic sort;
# 60 (180 rays <= 256): the threshold formed inside loss pass 2 (no median launch)
@pytest.mark.parametrize("mode,use_color,hd,n_per", [("mapper", True, False, 100), ("mapper", False, False, 100),
                                                     ("tracker", True, True, 100), ("tracker", False, True, 100),
                                                     ("tracker", True, False, 100), ("tracker", True, True, 400),
                                                     ("tracker", True, True, 60)])
def test_render_loss_matches_autograd(tiny, mode, use_color, hd, n_per):
    sc, frames = _frames(tiny)
    nice, c = _nice(sc)
    pix = torch.randint(96 * 128, (3 * n_per,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(4))
    ro, rd, gd, gc, keep = P.ops.gather_rays(frames, pix, n_per, 96, 128, (0, 96, 0, 128), sc.fx, sc.fy, sc.cx,
                                             sc.cy, sc.bound)
    z = P.ops.sample_z(ro, rd, gd, sc.bound, 32, 16)
    pts = ro[:, None, :] + rd[:, None, :] * z[:, :, None]
    with torch.no_grad():
        raw = nice(pts.reshape(-1, 3), c, stage="color", oob_bound=sc.bound)
    w = 0.2 if mode == "mapper" else 0.5
    depth, var, color, rl, g_raw = P.ops.render_loss(raw, z, gd, gc, keep, mode=mode, use_color=use_color,
                                                     handle_dynamic=hd, w_color=w)
    d2, v2, c2, loss_ref, g_ref = _autograd_loss(raw, z, gd, gc, keep, mode, use_color, hd, w)
    assert torch.equal(depth, d2) and torch.equal(var, v2) and torch.equal(color, c2)
    assert abs(float(rl.sum()) - float(loss_ref)) <= 1e-6 * max(1.0, abs(float(loss_ref)))
    assert float((g_raw - g_ref).abs().max()) <= 1e-6 * max(1.0, float(g_ref.abs().max()))


def test_fused_adam_matches_torch():
    g = torch.Generator(device=DEV).manual_seed(0)
    grid = torch.randn(1, 32, 5, 6, 7, device=DEV, generator=g).contiguous(memory_format=torch.channels_last_3d)
    w = torch.randn(33, 17, device=DEV, generator=g)
    b = torch.randn(17, device=DEV, generator=g)
    rows = torch.tensor([0, 3, 4, 17, 100, 209], dtype=torch.int32, device=DEV)
    # torch reference over the masked vector (Mapper.py:314-333 semantics)
    flat_rows = grid.permute(0, 2, 3, 4, 1).reshape(-1, 32)
    vg = flat_rows[rows.long()].clone().requires_grad_(True)
    w_ref, b_ref = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    opt_ref = torch.optim.Adam([{"params": [w_ref], "lr": 0.01}, {"params": [b_ref], "lr": 0.003},
                                {"params": [vg], "lr": 0.1}], foreach=False)
    grid_f, w_f, b_f = grid.clone(), w.clone(), b.clone()
    opt = P.ops.FusedAdam([{"params": [w_f], "lr": 0.01}, {"params": [b_f], "lr": 0.003},
                           {"params": [grid_f], "lr": 0.1, "rows": rows}])
    for it in range(6):
        gw = torch.randn(33, 17, device=DEV, generator=g)
        gb = torch.randn(17, device=DEV, generator=g) if it % 2 == 0 else None   # b skips odd steps
        ggrid = torch.randn_like(grid).contiguous(memory_format=torch.channels_last_3d)
        w_ref.grad, vg.grad = gw.clone(), ggrid.permute(0, 2, 3, 4, 1).reshape(-1, 32)[rows.long()].clone()
        b_ref.grad = gb.clone() if gb is not None else None
        opt_ref.step()
        grads = {w_f: gw, grid_f: ggrid}
        if gb is not None:
            grads[b_f] = gb
        opt.step(grads=grads)
    assert rel_l2(w_f, w_ref.detach()) < 1e-6
    assert rel_l2(b_f, b_ref.detach()) < 1e-6
    got_rows = grid_f.permute(0, 2, 3, 4, 1).reshape(-1, 32)
    assert rel_l2(got_rows[rows.long()], vg.detach()) < 1e-6
    untouched = torch.ones(got_rows.shape[0], dtype=torch.bool, device=DEV)
    untouched[rows.long()] = False
    assert torch.equal(got_rows[untouched], flat_rows[untouched])
    assert float(opt.state[b_f]["step"]) == 3.0 and float(opt.state[w_f]["step"]) == 6.0


@pytest.mark.parametrize("n_vox", [210, 30000])
def test_fused_adam_live_count_matches_exact_rows(n_vox):
    """ABI v19 n_live: a row-masked segment sized for a capacity (row list and Adam state for every voxel,
    compact gradient [capacity][32]) whose live count is a device word updates exactly what a segment of
    the live rows alone does — bit for bit — and nothing else; with a capacity far above the live count
    (30000 voxels: the launch is capped at 512 workgroups that stride the live rows) too."""
    g = torch.Generator(device=DEV).manual_seed(1)
    Z = n_vox // 42
    grid = torch.randn(1, 32, Z, 6, 7, device=DEV, generator=g).contiguous(memory_format=torch.channels_last_3d)
    nv = grid.shape[2] * 42
    live = torch.randperm(nv, device=DEV, generator=g)[: nv // 3].sort().values.to(torch.int32)
    k = live.numel()
    cap_rows = torch.full((nv,), 7, dtype=torch.int32, device=DEV)   # (entries past k: never read)
    cap_rows[:k] = live
    n_live = torch.tensor([k], dtype=torch.int64, device=DEV)
    ga, gb = grid.clone(), grid.clone()
    opt_a = P.ops.FusedAdam([{"params": [ga], "lr": 0.05, "rows": live}])
    opt_b = P.ops.FusedAdam([{"params": [gb], "lr": 0.05, "rows": cap_rows, "n_live": n_live}])
    for _ in range(4):
        comp = torch.randn(k, 32, device=DEV, generator=g)
        cap = torch.randn(nv, 32, device=DEV, generator=g)   # garbage past the live rows
        cap[:k] = comp
        opt_a.step(grads={ga: comp.clone()})
        opt_b.step(grads={gb: cap})
    assert torch.equal(ga, gb)
    assert torch.equal(opt_a.state[ga]["exp_avg"], opt_b.state[gb]["exp_avg"][: k * 32])
    assert float(opt_b.state[gb]["exp_avg"][k * 32:].abs().max()) == 0.0   # state past the live rows untouched


def test_engine_iteration_matches_autograd_path(tiny):
    sc, frames = _frames(tiny)
    nice, c = _nice(sc)
    nice_ref, c_ref = _nice(sc)
    eng = P.engine.MappingEngine(nice, c, sc.bound, 32, 16, device=DEV)
    n_per = 100
    pix = torch.randint(96 * 128, (3 * n_per,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(6))
    # engine gradients (no optimizer step: lr 0 would still move Adam state; use a throwaway opt)
    opt = P.ops.FusedAdam([{"params": [eng.decs["color"].param], "lr": 0.0}] +
                          [{"params": [c[k]], "lr": 0.0} for k in ("grid_middle", "grid_fine", "grid_color")])
    ray_loss, keep = eng.iteration("color", frames, pix, n_per, (96, 128), (sc.fx, sc.fy, sc.cx, sc.cy), opt)
    # autograd path on the same rays: Renderer.render_batch_ray on kept rays + the mapper loss
    ro, rd, gd, gc, kp = P.ops.gather_rays(frames, pix, n_per, 96, 128, (0, 96, 0, 128), sc.fx, sc.fy, sc.cx, sc.cy,
                                           sc.bound)
    k = kp.bool()
    gl = {kk: v.detach().clone().requires_grad_(True) for kk, v in c_ref.items()}
    for p in nice_ref.parameters():
        p.requires_grad_(False)
    for p in nice_ref.color_decoder.parameters():
        p.requires_grad_(True)
    r = P.Renderer(base_cfg(), None, sc.slam(base_cfg()))
    depth, unc, color = r.render_batch_ray(gl, nice_ref, rd[k], ro[k], DEV, "color", gt_depth=gd[k])
    m = gd[k] > 0
    loss = torch.abs(gd[k][m] - depth[m]).sum() + 0.2 * torch.abs(gc[k] - color).sum()
    loss.backward()
    assert abs(float(ray_loss.sum()) - float(loss)) <= 1e-6 * float(loss)
    for kk in ("grid_middle", "grid_fine", "grid_color"):
        assert rel_l2(eng.ggrad[kk], gl[kk].grad) < 1e-5, kk
    ref = torch.cat([p.grad.reshape(-1) for p in nice_ref.color_decoder.parameters()])
    assert rel_l2(eng.decs["color"].grad, ref) < 1e-5


def test_engine_compact_gradients_match_dense(tiny):
    """Frustum-compacted grid gradients (engine rows → voxel slot map, ABI v6) == the dense
    gradients on the selected rows, and the row-masked Adam over them updates the grids like the
    dense path (Mapper.py:314-333,394-401: only the masked vector is optimised)."""
    sc, frames = _frames(tiny)
    pix = torch.randint(96 * 128, (3 * 150,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(12))
    keys = ("grid_middle", "grid_fine", "grid_color")
    out = {}
    for compact in (False, True):
        nice, c = _nice(sc)
        g = torch.Generator(device=DEV).manual_seed(3)
        rows = {k: torch.nonzero(torch.rand(c[k].shape[2:].numel(), device=DEV, generator=g) < 0.4)
                .reshape(-1).to(torch.int32) for k in keys}
        eng = P.engine.MappingEngine(nice, c, sc.bound, 32, 16, device=DEV, rows=rows if compact else None)
        opt = P.ops.FusedAdam([{"params": [eng.decs["color"].param], "lr": 0.005}] +
                              [{"params": [c[k]], "lr": 0.005, "rows": rows[k]} for k in keys])
        gr = {}

        def snapshot(ks, dn):  # runs where the ray-sharded exchange would: after backward, before Adam
            for k in keys:
                gg = eng.ggrad[k]
                gr[k] = gg.clone() if compact else gg.permute(0, 2, 3, 4, 1).reshape(-1, 32)[rows[k].long()].clone()

        eng.iteration("color", frames, pix, 150, (96, 128), (sc.fx, sc.fy, sc.cx, sc.cy), opt, exchange=snapshot)
        if compact:  # Adam consumed (zeroed) the compact gradients: the next iteration needs no memset
            assert float(eng.gbuf.abs().sum()) == 0.0
        out[compact] = (gr, {k: c[k].detach().clone() for k in keys}, eng.decs["color"].param.detach().clone())
        if compact:
            assert eng.gbuf.numel() == sum(r.numel() for r in rows.values()) * 32
    for k in keys:
        assert float(out[False][0][k].abs().sum()) > 0, k
        assert rel_l2(out[True][0][k], out[False][0][k]) < 1e-6, k
        assert rel_l2(out[True][1][k], out[False][1][k]) < 1e-6, k
    assert rel_l2(out[True][2], out[False][2]) < 1e-6


def test_engine_loss_decreases(tiny):
    sc, frames = _frames(tiny)
    nice, c = _nice(sc)
    eng = P.engine.MappingEngine(nice, c, sc.bound, 32, 16, device=DEV)
    opt = P.ops.FusedAdam([{"params": [eng.decs["color"].param], "lr": 0.005}] +
                          [{"params": [c[k]], "lr": 0.005} for k in ("grid_middle", "grid_fine", "grid_color")])
    pix = torch.randint(96 * 128, (3 * 200,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(8))
    losses = []
    for _ in range(8):
        rl, _ = eng.iteration("color", frames, pix, 200, (96, 128), (sc.fx, sc.fy, sc.cx, sc.cy), opt)
        losses.append(float(rl.sum()))
    assert losses[-1] < losses[0]


def test_engine_prefetch_matches_serial(tiny):
    """iteration(prefetch=True): the next batch's gather + sampler run on a side stream during this
    iteration's render/backward.  The device draw stream is consumed in the same order, so after
    the same number of iterations the map equals the serial engine's (up to float-atomic order),
    and the kept-ray counter covers one batch ahead."""
    sc, frames = _frames(tiny)
    out = {}
    # (prefetch, its stream, one merged Adam): serial; the round-5 default (the prefetch on the mask-only
    # launch's stream, one Adam after both branches); round 4's (its own stream, per-branch Adam)
    variants = ((False, "lean", True), (True, "lean", True), (True, "own", False))
    for key in variants:
        pre, pst, merge = key
        nice, c = _nice(sc)
        eng = P.engine.MappingEngine(nice, c, sc.bound, 32, 16, device=DEV)
        eng.prefetch_stream, eng.adam_merge = pst, merge
        opt = P.ops.FusedAdam([{"params": [eng.decs["color"].param], "lr": 0.005}] +
                              [{"params": [c[k]], "lr": 0.005} for k in ("grid_middle", "grid_fine", "grid_color")])
        kept = torch.zeros(1, dtype=torch.int64, device=DEV)
        losses = []
        for _ in range(4):
            rl, _ = eng.iteration("color", frames, None, 150, (96, 128), (sc.fx, sc.fy, sc.cx, sc.cy), opt,
                                  seed=11, n_kept=kept, prefetch=pre)
            losses.append(rl.clone())
        torch.cuda.synchronize()
        out[key] = (losses, {k: v.detach().clone() for k, v in c.items()}, eng.decs["color"].param.detach().clone(),
                    int(kept), sorted(float(st["step"]) for st in opt.state.values()))
    ref = out[variants[0]]
    for key in variants[1:]:
        o = out[key]
        for a, b in zip(ref[0], o[0]):
            assert rel_l2(b, a) < 1e-5, key
        for k in ref[1]:
            assert rel_l2(o[1][k], ref[1][k]) < 1e-5, (key, k)
        assert rel_l2(o[2], ref[2]) < 1e-5, key
        assert o[3] >= ref[3] > 0, key  # prefetch has drawn (and counted) one batch more
        assert o[4] == ref[4] == [4.0] * 4, key


def test_engine_per_branch_adam_matches_single_adam(tiny):
    """One rank: each decoder branch updates its own grid's rows (and the colour decoder) on its
    own stream right after its backward.  The same iterations with ONE Adam call after all the
    branches (the path an all-reduce hook takes) must give the same map."""
    sc, frames = _frames(tiny)
    out = {}
    for single in (False, True):
        nice, c = _nice(sc)
        eng = P.engine.MappingEngine(nice, c, sc.bound, 32, 16, device=DEV)
        opt = P.ops.FusedAdam([{"params": [eng.decs["color"].param], "lr": 0.005}] +
                              [{"params": [c[k]], "lr": 0.005} for k in ("grid_middle", "grid_fine", "grid_color")])
        pix = torch.randint(96 * 128, (3 * 150,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(12))
        for _ in range(3):
            eng.iteration("color", frames, pix, 150, (96, 128), (sc.fx, sc.fy, sc.cx, sc.cy), opt,
                          allreduce=(lambda grads: None) if single else None)
        torch.cuda.synchronize()
        out[single] = ({k: v.detach().clone() for k, v in c.items()}, eng.decs["color"].param.detach().clone(),
                       {id(p): float(st["step"]) for p, st in opt.state.items()})
    for k in out[False][0]:
        assert rel_l2(out[True][0][k], out[False][0][k]) < 1e-5, k
    assert rel_l2(out[True][1], out[False][1]) < 1e-5
    assert sorted(out[True][2].values()) == sorted(out[False][2].values()) == [3.0] * 4


def test_engine_branch_order_and_concurrency_keep_the_map(tiny):
    """ABI v16: the colour decoder's weight gradients (nslam_color_wgrad) run beside the lean backward
    of every decoder.  Enqueued first or second, on concurrent streams or one: three iterations give
    the same map, decoder, packed copy and Adam steps (grid atomics order aside)."""
    sc, frames = _frames(tiny)
    out = {}
    for variant in ("first", "second", "serial"):
        nice, c = _nice(sc)
        eng = P.engine.MappingEngine(nice, c, sc.bound, 32, 16, device=DEV)
        eng.wgrad_first = variant != "second"
        eng.concurrent = variant != "serial"
        opt = P.ops.FusedAdam([{"params": [eng.decs["color"].param], "lr": 0.005}] +
                              [{"params": [c[k]], "lr": 0.005} for k in ("grid_middle", "grid_fine", "grid_color")])
        for it in range(3):
            pix = torch.randint(96 * 128, (3 * 150,), device=DEV,
                                generator=torch.Generator(device=DEV).manual_seed(20 + it))
            eng.iteration("color", frames, pix, 150, (96, 128), (sc.fx, sc.fy, sc.cx, sc.cy), opt)
        torch.cuda.synchronize()
        out[variant] = ({k: v.detach().clone() for k, v in c.items()}, eng.decs["color"].param.detach().clone(),
                        eng.decs["color"].packed.clone(), sorted(float(st["step"]) for st in opt.state.values()))
    b = out["serial"]
    for v in ("first", "second"):
        a = out[v]
        for k in a[0]:
            assert rel_l2(a[0][k], b[0][k]) < 1e-5, (v, k)
        assert rel_l2(a[1], b[1]) < 1e-5 and rel_l2(a[2], b[2]) < 1e-5, v
        assert a[3] == b[3] == [3.0] * 4, v


@pytest.mark.parametrize("n_rays", [150, 1000, 3333])
def test_color_wgrad_matches_recompute_backward(tiny, n_rays):
    """k_color_wgrad (the split-K weight gradients from the activation tape, ABI v16) vs the colour
    decoder's recompute backward (k_dec_bwd with weight gradients: forward recomputed, LDS transposes,
    per-tile slabs) on the same rays and cotangent, ELEMENTWISE over every colour-decoder parameter —
    the two share no weight-gradient code.  Ragged batches (n not a multiple of 32), one and several
    tiles per chunk (150 rays: 1 tile per chunk; 3333 rays x 48: 5 tiles per chunk)."""
    sc, frames = _frames(tiny)
    nice, c = _nice(sc)
    eng = P.engine.MappingEngine(nice, c, sc.bound, 32, 16, device=DEV)
    g = torch.Generator(device=DEV).manual_seed(30 + n_rays)
    pix = torch.randint(96 * 128, (n_rays,), device=DEV, generator=g)
    ro, rd, gd, gc, keep = P.ops.gather_rays(frames[:1], pix, n_rays, 96, 128, (0, 96, 0, 128), sc.fx, sc.fy, sc.cx,
                                             sc.cy)
    z = P.ops.sample_z(ro, rd, gd, sc.bound, 32, 16)
    n = z.numel()
    eng.query_fwd("color", ro, rd, z, tape=True)
    g_raw = torch.randn(n, 4, device=DEV, generator=g)
    cfg = eng._cfg("color", ro, rd, z, (), ("color",))
    dgrad = eng.decs["color"].grad
    res = {}
    for path in ("tape", "recompute"):
        dgrad.zero_()
        cfg.act_tape = eng._tape.data_ptr() if path == "tape" else None
        cfg.saved_masks = eng._saved.data_ptr() if path == "tape" else None
        wsb = P._lib.lib().nslam_query_bwd_decoder_workspace_size(ctypes.byref(cfg), P._lib.DEC_COLOR, n)
        ws = torch.empty(wsb, dtype=torch.uint8, device=DEV)
        if path == "tape":
            rc = P._lib.lib().nslam_color_wgrad(ctypes.byref(cfg), None, n, g_raw.data_ptr(), ws.data_ptr(), wsb,
                                                torch.cuda.current_stream().cuda_stream)
        else:
            rc = P._lib.lib().nslam_query_bwd_decoder(ctypes.byref(cfg), P._lib.DEC_COLOR, 0, None, n,
                                                      g_raw.data_ptr(), None, ws.data_ptr(), wsb,
                                                      torch.cuda.current_stream().cuda_stream)
        assert rc == 0, (path, rc)
        torch.cuda.synchronize()
        res[path] = dgrad.clone()
    a, b = res["tape"], res["recompute"]
    assert float(b.abs().sum()) > 0
    assert rel_l2(a, b) < 1e-5
    # elementwise, on every parameter tensor (a mis-placed block would show as a large local error)
    for name, t_a, t_b in zip(eng.decs["color"].packer.names, eng.decs["color"].packer.split_grad(a),
                              eng.decs["color"].packer.split_grad(b)):
        scale = float(t_b.abs().max()) + 1e-30
        err = float((t_a - t_b).abs().max()) / scale
        assert err < 1e-4, (name, err)


def test_rows_pack_unpack_bitexact():
    """nslam_rows_pack / nslam_rows_unpack (the sparse gradient exchange) vs torch indexing."""
    g = torch.Generator(device=DEV).manual_seed(9)
    grid = torch.randn(5000 * 32, device=DEV, generator=g)
    rows = torch.randperm(5000, device=DEV, generator=g)[:1234].to(torch.int32)
    tail = torch.randn(1001, device=DEV, generator=g)
    buf = torch.full((1234 * 32 + 1001 + 3,), float("nan"), device=DEV)
    P.ops.rows_pack(grid, rows, None, buf)
    P.ops.rows_pack(None, None, tail, buf[1234 * 32:1234 * 32 + 1001])
    torch.cuda.synchronize()
    assert torch.equal(buf[:1234 * 32].view(-1, 32), grid.view(-1, 32)[rows.long()])
    assert torch.equal(buf[1234 * 32:1234 * 32 + 1001], tail)
    buf2 = torch.randn(buf.shape, device=DEV, generator=g)
    grid2, tail2 = grid.clone(), tail.clone()
    P.ops.rows_unpack(buf2, rows, grid2, None)
    P.ops.rows_unpack(buf2[1234 * 32:1234 * 32 + 1001], None, None, tail2)
    torch.cuda.synchronize()
    ref = grid.clone().view(-1, 32)
    ref[rows.long()] = buf2[:1234 * 32].view(-1, 32)
    assert torch.equal(grid2.view(-1, 32), ref)
    assert torch.equal(tail2, buf2[1234 * 32:1234 * 32 + 1001])


def test_sparse_exchange_single_rank_is_identity(tiny):
    """world size 1 (no process group): the frustum-compacted exchange (pack → [no collective] →
    unpack) leaves an engine iteration's gradients bit-identical."""
    sc, frames = _frames(tiny)
    pix = torch.randint(96 * 128, (3 * 100,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(6))
    nice, c = _nice(sc)
    eng = P.engine.MappingEngine(nice, c, sc.bound, 32, 16, device=DEV)
    opt = P.ops.FusedAdam([{"params": [eng.decs["color"].param], "lr": 0.0}] +
                          [{"params": [c[k]], "lr": 0.0} for k in ("grid_middle", "grid_fine", "grid_color")])
    eng.iteration("color", frames, pix, 100, (96, 128), (sc.fx, sc.fy, sc.cx, sc.cy), opt)
    rows = {k: torch.arange(0, c[k].shape[2:].numel(), 3, device=DEV, dtype=torch.int32)
            for k in ("grid_middle", "grid_fine", "grid_color")}
    ex = P.distributed.SparseGradExchange(eng, rows)
    keys, dn = eng.grads_for("color", ("color",))
    g0, d0 = eng.gbuf.clone(), eng.decs["color"].grad.clone()
    assert float(g0.abs().sum()) > 0 and float(d0.abs().sum()) > 0
    ex(keys, dn)
    torch.cuda.synchronize()
    assert torch.equal(eng.gbuf, g0) and torch.equal(eng.decs["color"].grad, d0)
    assert ex.payload_bytes(keys, dn) == (sum(r.numel() for r in rows.values()) * 32 + d0.numel()) * 4


@pytest.mark.parametrize("stage", ["fine", "color"])
@pytest.mark.parametrize("n_per", [13, 1400])
def test_forward_variants_bitexact(tiny, stage, n_per):
    """Every nslam_query_fwd_ws variant (ABI v18 fwd_variant: one-wave units, the persistent producer /
    consumer workgroups, 4-wave parts) forms the same values in the same order: raw, the saved ReLU
    masks and the colour decoder's activation tape are bit-identical.  3 x 1400 rays x 48 samples =
    6300 tiles, ~74 decoder units per CU: the producer / consumer ring wraps ~10 times; 3 x 13 rays: a
    partial last tile and fewer units than CUs."""
    sc, frames = _frames(tiny)
    nice, c = _nice(sc)
    eng = P.engine.MappingEngine(nice, c, sc.bound, 32, 16, device=DEV)
    g = torch.Generator(device=DEV).manual_seed(5)
    pix = torch.randint(96 * 128, (3 * n_per,), device=DEV, generator=g)
    ro, rd, gd, gc, keep = P.ops.gather_rays(frames, pix, n_per, 96, 128, (0, 96, 0, 128), sc.fx, sc.fy, sc.cx,
                                             sc.cy)
    z = P.ops.sample_z(ro, rd, gd, sc.bound, 32, 16)
    outs = {}
    for v in (P.ops.FWD_UNITS, P.ops.FWD_PC, P.ops.FWD_PARTS):
        P.ops.FWD_VARIANT = v
        try:
            raw = eng.query_fwd(stage, ro, rd, z, tape=True)
            torch.cuda.synchronize()
            outs[v] = (raw.clone(), eng._saved.clone(), None if eng._tape is None else eng._tape.clone())
        finally:
            P.ops.FWD_VARIANT = P.ops.FWD_DEFAULT
    ref = outs[P.ops.FWD_UNITS]
    assert bool(torch.isfinite(ref[0]).all())
    ntiles = (z.numel() + 31) // 32
    decs = [1, 2, 3] if stage == "color" else [1, 2]  # the masks the stage writes: [decoder][tile][5][64]
    for v, o in outs.items():
        assert torch.equal(o[0], ref[0]), v
        m, mr = (x.view(torch.int16).view(4, ntiles, 5, 64)[decs] for x in (o[1], ref[1]))
        assert torch.equal(m, mr), v
        if stage == "color":
            assert torch.equal(o[2], ref[2]), v


@pytest.mark.parametrize("stage", ["middle", "fine", "color"])
def test_decoder_parallel_forward_bitexact(tiny, stage):
    """nslam_query_fwd_ws (one decoder per workgroup + occupancy combine) == nslam_query_fwd
    (every decoder in one wave), raw and saved ReLU masks, pts form incl. out-of-bound points."""
    sc, frames = _frames(tiny)
    nice, c = _nice(sc)
    g = torch.Generator(device=DEV).manual_seed(11)
    lo, hi = sc.bound[:, 0].to(DEV), sc.bound[:, 1].to(DEV)
    pts = (lo - 0.2 + (hi - lo + 0.4) * torch.rand(3001, 3, device=DEV, dtype=torch.float64, generator=g))
    outs = []
    for split in (False, True):
        P.ops.SPLIT_FWD = split
        try:
            with torch.enable_grad():
                gl = {k: v.detach().clone().requires_grad_(True) for k, v in c.items()}
                raw = nice(pts, gl, stage=stage, oob_bound=sc.bound)
            outs.append(raw.detach().clone())
        finally:
            P.ops.SPLIT_FWD = True
    inside = ((pts > lo) & (pts < hi)).all(1)
    assert bool((~inside).any()) and bool(inside.any())
    assert torch.equal(outs[0], outs[1])


def test_tracking_engine_matches_oracle(tiny):
    """TrackingEngine (fused camera iteration, Tracker.py:71-128) vs the oracle's autograd replica on
    the same pixel draws: per-iteration losses, first camera gradient, camera after 3 steps."""
    import copy

    from test_gpu_dropins import oracle_samples
    sc = Scene(tiny)
    slam = sc.slam(base_cfg())
    eng = P.engine.TrackingEngine(copy.deepcopy(slam.shared_decoders), slam.shared_c, sc.bound, 32, 16,
                                  (sc.H, sc.W), (sc.fx, sc.fy, sc.cx, sc.cy), ignore_edge=(20, 20), w_color=0.5,
                                  handle_dynamic=True, use_color=True, device=DEV)
    cam0 = P.common.get_tensor_from_camera(sc.c2w).cuda()
    cam = cam0.clone().requires_grad_(True)
    opt = P.ops.FusedAdam([{"params": [cam], "lr": 0.001}])
    g = torch.Generator().manual_seed(11)
    pixs = [torch.randint(eng.n_window(), (200,), generator=g) for _ in range(3)]
    losses, grads = [], []
    for k in range(3):
        losses.append(float(eng.iteration(cam, sc.depth.cuda(), sc.color.cuda(), pixs[k].cuda(), opt)))
        grads.append(cam.grad.detach().clone())
    camo = cam0.cpu().clone().requires_grad_(True)
    opto = torch.optim.Adam([camo], lr=0.001)
    ref, ref_grads = [], []
    for k in range(3):
        opto.zero_grad()
        c2w = orc.camera_from_tensor(camo)
        ro, rd, gd, gc = oracle_samples(sc, pixs[k], 20, sc.H - 20, 20, sc.W - 20, c2w, sc.depth, sc.color)
        keep = orc.inside_mask(ro, rd, gd, sc.bound)
        ro, rd, gd, gc = ro[keep], rd[keep], gd[keep], gc[keep]
        d, v, c = orc.render_batch_ray(sc.sd, sc.grids, rd, ro, "color", sc.bound, gd)
        loss = orc.tracker_loss(d, v, c, gd, gc)
        loss.backward()
        ref_grads.append(camo.grad.detach().clone())
        opto.step()
        ref.append(float(loss))
    np.testing.assert_allclose(losses, ref, rtol=2e-4)
    assert rel_l2(grads[0], ref_grads[0]) < 1e-3
    assert rel_l2(cam.detach().cpu() - cam0.cpu(), camo.detach() - cam0.cpu()) < 1e-2


def test_cam_grad_parts_matches_single_workgroup(tiny):
    """ABI v15 nslam_cam_grad_parts (decoder d/dpts shares summed in the kernel, several workgroups
    meeting through a ticket) == the torch adds + single-workgroup nslam_cam_grad, up to the order of
    the float64 partial sums; repeated calls reuse the re-armed ticket."""
    import copy
    sc = Scene(tiny)
    slam = sc.slam(base_cfg())
    cam0 = P.common.get_tensor_from_camera(sc.c2w).cuda()
    pix = torch.randint(400, (200,), generator=torch.Generator().manual_seed(9))
    out = {}
    for parts in (True, False):
        te = P.engine.TrackingEngine(copy.deepcopy(slam.shared_decoders), slam.shared_c, sc.bound, 32, 16,
                                     (sc.H, sc.W), (sc.fx, sc.fy, sc.cx, sc.cy), ignore_edge=(20, 20), w_color=0.5,
                                     handle_dynamic=True, use_color=True, device=DEV)
        te.cam_parts = parts
        cam = cam0.clone().requires_grad_(True)
        opt = P.ops.FusedAdam([{"params": [cam], "lr": 0.0}])
        gs = []
        for _ in range(3):  # lr 0: the same pose, the same draws -> the same gradient every call
            te.iteration(cam, sc.depth.cuda(), sc.color.cuda(), (pix % te.n_window()).cuda(), opt)
            gs.append(cam.grad.detach().clone())
        out[parts] = gs
    assert float(out[False][0].abs().sum()) > 0
    for a, b in zip(out[True], out[False]):
        assert rel_l2(a, b) < 1e-6
    assert torch.equal(out[True][0], out[True][1]) and torch.equal(out[True][1], out[True][2])


def test_tracker_track_frame_fused_matches_loop(tiny):
    """Tracker.track_frame on the TrackingEngine == the reference loop over optimize_cam_in_batch
    (same generator ⇒ same pixel draws; device-side best-pose selection vs loss.item())."""
    cfg = base_cfg()
    sc = Scene(tiny)
    outs = []
    for fused in (False, True):
        slam = sc.slam(cfg)
        tr = P.Tracker(cfg, None, slam, generator=torch.Generator(device=DEV).manual_seed(4))
        tr.fused = fused
        c2w = torch.cat([sc.c2w, torch.tensor([[0, 0, 0, 1.0]])], 0).cuda()
        pre = c2w.clone()
        pre[:3, 3] += 0.02
        outs.append(tr.track_frame(1, sc.color.cuda(), sc.depth.cuda(), c2w, pre_c2w=pre))
    assert torch.allclose(outs[0], outs[1], atol=5e-4), (outs[0] - outs[1]).abs().max()


def test_sampler_batch_max_paths_agree(tiny):
    """The sampler's batch-global max(gt_depth) (Renderer.py:107-111,144) three ways — reduced
    inside the sampling kernel (small batches), by a separate k_max_gt pass (large batches) and
    given by the caller (ray sharding) — yields bit-identical z_vals."""
    sc, frames = _frames(tiny)
    g = torch.Generator(device=DEV).manual_seed(21)
    for n in (700, 9000):
        ro = (sc.bound[:, 0] + 0.5 * (sc.bound[:, 1] - sc.bound[:, 0])).float().to(DEV).expand(n, 3).contiguous()
        rd = torch.randn(n, 3, device=DEV, generator=g)
        gd = torch.rand(n, device=DEV, generator=g) * 2.0
        gd[::7] = 0.0
        z0 = P.ops.sample_z(ro, rd, gd, sc.bound, 32, 16)
        z1 = P.ops.sample_z(ro, rd, gd, sc.bound, 32, 16, gt_max=gd.max().reshape(1))
        assert torch.equal(z0, z1), n
        # a shard given the full batch's max samples exactly as the full batch does
        zs = P.ops.sample_z(ro[:100], rd[:100], gd[:100], sc.bound, 32, 16, gt_max=gd.max().reshape(1))
        assert torch.equal(zs, z0[:100]), n


def _mix64(x):
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
    return x ^ (x >> np.uint64(31))


def _drawn_pix(seed, ctr, n, wn):
    """Host restatement of nslam_gather_rays' in-kernel draws (ABI v7, splitmix64 + Lemire)."""
    with np.errstate(over="ignore"):
        r = np.arange(n, dtype=np.uint64)
        h = _mix64(np.uint64(seed) ^ _mix64(np.uint64(ctr) * np.uint64(0x9e3779b97f4a7c15) + r))
        return ((h >> np.uint64(32)) * np.uint64(wn)) >> np.uint64(32)


@pytest.mark.parametrize("window", [(0, 96, 0, 128), (20, 76, 20, 108)])
def test_gather_rays_device_draws(tiny, window):
    """pix=None draws select_uv's indices inside the kernel: the rays equal an explicit-pix gather of
    the host-restated draws bit for bit, the counter advances once per call, n_kept counts keep."""
    sc, frames = _frames(tiny)
    H, W = 96, 128
    h0, h1, w0, w1 = window
    wn = (h1 - h0) * (w1 - w0)
    n_per = 700
    draw = P.ops.PixelDraws(1234, DEV)
    kept = torch.zeros(1, dtype=torch.int64, device=DEV)
    seen = []
    for call in range(3):
        out = P.ops.gather_rays(frames, None, n_per, H, W, window, sc.fx, sc.fy, sc.cx, sc.cy, sc.bound,
                                draw=draw, n_kept=kept)
        assert int(draw.counter) == call + 1
        pix = torch.from_numpy(_drawn_pix(1234, call, len(frames) * n_per, wn).astype(np.int64)).to(DEV)
        ref = P.ops.gather_rays(frames, pix, n_per, H, W, window, sc.fx, sc.fy, sc.cx, sc.cy, sc.bound)
        for a, b in zip(out, ref):
            assert torch.equal(a, b)
        seen.append(pix)
        assert int(draw.ticket) == 0
    assert int(kept) == sum(int(P.ops.gather_rays(frames, p, n_per, H, W, window, sc.fx, sc.fy, sc.cx, sc.cy,
                                                      sc.bound)[4].sum()) for p in seen)
    allp = torch.cat(seen).cpu().numpy()
    assert allp.min() >= 0 and allp.max() < wn
    # uniform over the window: each quarter of the window index range gets 25% +- 3%
    q = np.bincount(allp * 4 // wn, minlength=4) / allp.size
    assert np.all(np.abs(q - 0.25) < 0.03), q


def test_gather_rays_from_camera_vectors(tiny):
    """ABI v21 nslam_frame.cam: frames given by their camera 7-vectors — the gather forms each pose itself
    (nslam_cam_pose's arithmetic) and writes it to c2w_out: the pose equals nslam_cam_pose's bit for bit
    and the rays equal a gather of frames given by that pose; frames of both kinds mix in one call."""
    sc, frames = _frames(tiny)
    H, W = 96, 128
    g = torch.Generator().manual_seed(3)
    cams = []
    for f in range(len(frames)):
        q = torch.randn(4, generator=g)
        cams.append(torch.cat([q / q.norm(), torch.randn(3, generator=g) * 0.3]).float().to(DEV))
    poses = [P.ops.cam_pose(c, torch.empty(3, 4, dtype=torch.float32, device=DEV)) for c in cams]
    outs = [torch.full((3, 4), -7.0, dtype=torch.float32, device=DEV) for _ in cams]
    mixed = [(d, c, outs[f], cams[f]) if f != 1 else (d, c, poses[f]) for f, (d, c, _) in enumerate(frames)]
    ref_frames = [(d, c, poses[f]) for f, (d, c, _) in enumerate(frames)]
    pix = torch.randint(H * W, (len(frames) * 300,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(4))
    got = P.ops.gather_rays(mixed, pix, 300, H, W, (0, H, 0, W), sc.fx, sc.fy, sc.cx, sc.cy, sc.bound)
    ref = P.ops.gather_rays(ref_frames, pix, 300, H, W, (0, H, 0, W), sc.fx, sc.fy, sc.cx, sc.cy, sc.bound)
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
    for f in (0, 2):
        assert torch.equal(outs[f], poses[f])
    assert bool((outs[1] == -7.0).all())  # a frame given by its pose: nothing written


def test_adam_mirror_keeps_packed_copy_current(tiny):
    """FusedAdam.set_mirror: the engine's packed decoder copy after Adam equals a fresh repack."""
    sc, frames = _frames(tiny)
    nice, c = _nice(sc)
    eng = P.engine.MappingEngine(nice, c, sc.bound, 32, 16, device=DEV)
    opt = P.ops.FusedAdam([{"params": [eng.decs["color"].param], "lr": 0.005}] +
                          [{"params": [c[k]], "lr": 0.005} for k in ("grid_middle", "grid_fine", "grid_color")])
    pix = torch.randint(96 * 128, (3 * 150,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(3))
    for _ in range(2):
        eng.iteration("color", frames, pix, 150, (96, 128), (sc.fx, sc.fy, sc.cx, sc.cy), opt)
    d = eng.decs["color"]
    assert d.param in opt.mirrors
    got = d.packed.clone()
    d.repack()
    assert torch.equal(got, d.packed)


def test_sharded_draws_slice_the_global_batch(tiny):
    """Ray sharding without a collective: rank r of `world` (same seed) gathers exactly its slice of
    the global batch (n_per*world pixels per frame), its gather kernel reports the global batch's
    max(gt_depth) over kept rays, and its z-values equal the global batch's (Renderer.py:107-111,144)."""
    sc, frames = _frames(tiny)
    H, W, n_per, world = 96, 128, 300, 3
    args = (H, W, (0, H, 0, W), sc.fx, sc.fy, sc.cx, sc.cy, sc.bound)
    full = P.ops.gather_rays(frames, None, n_per * world, *args, draw=P.ops.PixelDraws(77, DEV))
    z_full = P.ops.sample_z(full[0], full[1], full[2], sc.bound, 32, 16)
    nf = len(frames)
    for rank in range(world):
        dr = P.ops.PixelDraws(77, DEV, world, rank, with_max=True)
        for it in range(2):  # the key re-arms itself: a second call reports the same max
            out = P.ops.gather_rays(frames, None, n_per, *args, draw=dr)
            dr.counter.zero_()
            assert float(dr.gt_max) == float(full[2].max()), (rank, it)
            assert int(dr.key) == 0 and int(dr.ticket) == 0
        sl = torch.cat([torch.arange(f * n_per * world + rank * n_per, f * n_per * world + (rank + 1) * n_per)
                        for f in range(nf)]).to(DEV)
        for a, b in zip(out, full):
            assert torch.equal(a, b[sl])
        z = P.ops.sample_z(out[0], out[1], out[2], sc.bound, 32, 16, gt_max=dr.gt_max)
        assert torch.equal(z, z_full[sl])


def test_cam_grad_kernel_matches_autograd():
    """nslam_cam_grad (ABI v9) vs autograd through get_camera_from_tensor and pts = t + (R·dir)·z;
    the pose handed to the kernel is get_camera_from_tensor's own (common.py:163-176)."""
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(4)
    for n in (1, 200, 777):
        cam = torch.randn(7, generator=g)
        S = 48
        z = torch.rand(n, S, generator=g, dtype=torch.float64) * 3
        dirs = torch.randn(n, 3, generator=g)
        camg = cam.clone().requires_grad_(True)
        R = P.common.get_camera_from_tensor(camg)
        rd = (dirs[:, None, :] * R[:3, :3]).sum(-1)
        pts = R[:3, 3][None, None, :].double() + rd[:, None, :].double() * z[..., None]
        gpts = torch.randn(n * S, 3, generator=g, dtype=torch.float64)
        (ref,) = torch.autograd.grad(pts.reshape(-1, 3), camg, gpts)
        c2w = P.common.get_camera_from_tensor(cam.to(dev))
        out = torch.empty(7, device=dev)
        P.ops.cam_grad(cam.to(dev), c2w.contiguous(), gpts.to(dev), z.to(dev), rd.detach().to(dev).contiguous(), out)
        assert float((out.cpu() - ref).norm() / ref.norm()) < 1e-5, n


def test_cam_pose_kernel_matches_get_camera_from_tensor():
    """nslam_cam_pose (ABI v9) vs the torch restatement of get_camera_from_tensor on the device.
    Same products and differences; |q|² may be summed in a different order than torch's reduce,
    so the pose is checked to 2 ulp-scale (rel 1e-6), and the exact-match fraction is reported."""
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(6)
    exact, worst = 0, 0.0
    out = torch.empty(3, 4, device=dev)
    for _ in range(200):
        cam = torch.randn(7, generator=g).to(dev)
        ref = P.common.get_camera_from_tensor(cam)
        P.ops.cam_pose(cam, out)
        exact += bool(torch.equal(out, ref))
        worst = max(worst, float((out - ref).abs().max() / ref.abs().max()))
    print(f"cam_pose: {exact}/200 bit-identical, worst rel {worst:.2e}")
    assert worst < 1e-6


@pytest.mark.gpu
def test_merged_backward_matches_per_decoder_launches(tiny):
    """ABI v10/v16: every decoder's mask-only backward as ONE launch beside the colour weight
    gradients (nslam_query_bwd_decoders + nslam_color_wgrad, the engine's two branches) == one
    nslam_query_bwd_decoder launch per decoder (the library running the colour tape backward's two
    kernels in sequence): mapping grid gradients (float atomics: up to summation order), the colour
    decoder's gradient (the same kernels: bit-exact) and the tracking camera gradient (per-decoder
    d/dpts buffers: bit-exact)."""
    import copy

    sc, frames = _frames(tiny)
    keys = ("grid_middle", "grid_fine", "grid_color")
    pix = torch.randint(96 * 128, (3 * 150,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(21))
    out = {}
    for merge in (False, True):
        nice, c = _nice(sc)
        eng = P.engine.MappingEngine(nice, c, sc.bound, 32, 16, device=DEV)
        eng.merge = merge
        opt = P.ops.FusedAdam([{"params": [eng.decs["color"].param], "lr": 0.0}] +
                              [{"params": [c[k]], "lr": 0.0} for k in keys])
        gr = {}

        def snapshot(ks, dn):
            for k in keys:
                gr[k] = eng.ggrad[k].clone()
            gr["dec"] = eng.decs["color"].grad.clone()

        eng.iteration("color", frames, pix, 150, (96, 128), (sc.fx, sc.fy, sc.cx, sc.cy), opt, exchange=snapshot)
        out[merge] = gr
    for k in keys:
        assert float(out[False][k].abs().sum()) > 0, k
        assert rel_l2(out[True][k], out[False][k]) < 1e-6, k
    assert torch.equal(out[True]["dec"], out[False]["dec"])
    # tracking: middle, fine and colour frozen, d/dpts per decoder
    scn = Scene(tiny)
    slam = scn.slam(base_cfg())
    cam0 = P.common.get_tensor_from_camera(scn.c2w).cuda()
    pixs = torch.randint(400, (200,), generator=torch.Generator().manual_seed(5))
    grads = {}
    for merge in (False, True):
        te = P.engine.TrackingEngine(copy.deepcopy(slam.shared_decoders), slam.shared_c, scn.bound, 32, 16,
                                     (scn.H, scn.W), (scn.fx, scn.fy, scn.cx, scn.cy), ignore_edge=(20, 20),
                                     w_color=0.5, handle_dynamic=True, use_color=True, device=DEV)
        te.eng.merge = merge
        cam = cam0.clone().requires_grad_(True)
        opt = P.ops.FusedAdam([{"params": [cam], "lr": 0.0}])
        te.iteration(cam, scn.depth.cuda(), scn.color.cuda(), (pixs % te.n_window()).cuda(), opt)
        grads[merge] = cam.grad.detach().clone()
    assert float(grads[False].abs().sum()) > 0
    assert torch.equal(grads[True], grads[False])


def test_engine_prefetch_discards_batch_of_other_frames(tiny):
    """A prefetched batch belongs to the frames it was gathered from: a call with another keyframe
    window (or with poses changed in place) draws its own batch from its own frames."""
    sc, frames = _frames(tiny)
    nice, c = _nice(sc)
    eng = P.engine.MappingEngine(nice, c, sc.bound, 32, 16, device=DEV)
    opt = P.ops.FusedAdam([{"params": [eng.decs["color"].param], "lr": 0.005}] +
                          [{"params": [c[k]], "lr": 0.005} for k in ("grid_middle", "grid_fine", "grid_color")])
    args = (None, 150, (96, 128), (sc.fx, sc.fy, sc.cx, sc.cy), opt)
    eng.iteration("color", frames, *args, seed=11, prefetch=True)
    moved = [(d, col, m.clone()) for d, col, m in frames]
    for f, (_, _, m) in enumerate(moved):
        m[:3, 3] += 0.05 * (f + 1)
    eng.iteration("color", moved, *args, seed=11, prefetch=True)   # another window: fresh batch (set 0)
    ro = eng._pre[2][0][0].view(len(moved), 150, 3)
    for f, (_, _, m) in enumerate(moved):
        assert torch.equal(ro[f], m[:3, 3].expand(150, 3)), f
    with torch.no_grad():
        moved[0][2][:3, 3] += 0.01                                     # a pose updated in place
    eng.iteration("color", moved, *args, seed=11, prefetch=True)
    ro = eng._pre[2][0][0].view(len(moved), 150, 3)
    assert torch.equal(ro[0], moved[0][2][:3, 3].expand(150, 3))


@pytest.mark.parametrize("with_best", [False, True])
def test_cam_grad_step_matches_separate_launches(tiny, with_best):
    """nslam_cam_grad_step (ABI v23): the tracking iteration with the camera's Adam step, the loss sum and the
    best-pose update fused into the camera-gradient launch == cam_grad_parts + FusedAdam.step + loss_sum_best,
    bit for bit over 6 iterations (camera, gradient, Adam moments and step count, loss, best pose and loss)."""
    import copy
    scn = Scene(tiny)
    slam = scn.slam(base_cfg())
    cam0 = P.common.get_tensor_from_camera(scn.c2w).cuda()
    cam0[4:] += torch.tensor([0.02, -0.01, 0.015], device=DEV)
    gen = torch.Generator().manual_seed(9)
    pixs = [torch.randint(400, (200,), generator=gen) for _ in range(6)]
    runs = {}
    for tail in (False, True):
        te = P.engine.TrackingEngine(copy.deepcopy(slam.shared_decoders), slam.shared_c, scn.bound, 32, 16,
                                     (scn.H, scn.W), (scn.fx, scn.fy, scn.cx, scn.cy), ignore_edge=(20, 20),
                                     w_color=0.5, handle_dynamic=True, use_color=True, device=DEV)
        te.cam_tail = tail
        cam = cam0.clone().requires_grad_(True)
        opt = P.ops.FusedAdam([{"params": [cam], "lr": 0.003}])
        best = (torch.full((), float("inf"), dtype=torch.float64, device=DEV), cam0.clone()) if with_best else None
        trace = []
        for pix in pixs:
            loss = te.iteration(cam, scn.depth.cuda(), scn.color.cuda(), (pix % te.n_window()).cuda(), opt, best=best)
            trace.append(torch.cat([cam.detach(), cam.grad.detach(), *opt.state_of(cam)]).clone())
            trace.append(loss.detach().clone().view(1))
        if best is not None:
            trace += [best[0].clone().view(1), best[1].clone()]
        runs[tail] = trace
    assert float(runs[False][1].abs().sum()) > 0
    assert not torch.equal(runs[False][0][:7], cam0)  # the camera moved
    for a, b in zip(runs[True], runs[False]):
        assert torch.equal(a, b), (a - b).abs().max()


@pytest.mark.parametrize("n_per,nan", [(60, False), (60, True), (85, False), (2, False)])
def test_tracker_median_in_pass2_matches_median_launch(tiny, monkeypatch, n_per, nan):
    """Up to 256 rays the tracker loss's handle_dynamic threshold is formed inside loss pass 2 by every
    workgroup (rank selection; the bitonic sort with a NaN residual) instead of the k_median_thr launch:
    the same outputs bit for bit (NaN where NaN) — NSLAM_MEDIAN_LAUNCH=1 forces the launch."""
    sc, frames = _frames(tiny)
    nice, c = _nice(sc)
    pix = torch.randint(96 * 128, (3 * n_per,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(8))
    ro, rd, gd, gc, keep = P.ops.gather_rays(frames, pix, n_per, 96, 128, (0, 96, 0, 128), sc.fx, sc.fy, sc.cx,
                                             sc.cy, sc.bound)
    z = P.ops.sample_z(ro, rd, gd, sc.bound, 32, 16)
    pts = ro[:, None, :] + rd[:, None, :] * z[:, :, None]
    with torch.no_grad():
        raw = nice(pts.reshape(-1, 3), c, stage="color", oob_bound=sc.bound).reshape(z.shape[0], z.shape[1], 4)
    if nan:
        k = int(torch.nonzero(keep)[0])
        raw[k, :, 3] = float("nan")
    outs = {}
    for launch in (False, True):
        if launch:
            monkeypatch.setenv("NSLAM_MEDIAN_LAUNCH", "1")
        outs[launch] = P.ops.render_loss(raw, z, gd, gc, keep, mode="tracker", use_color=True, handle_dynamic=True,
                                         w_color=0.5)
    for a, b in zip(outs[False], outs[True]):
        torch.testing.assert_close(a, b, rtol=0, atol=0, equal_nan=True)
    assert float(outs[False][3].nan_to_num().abs().sum()) > 0
