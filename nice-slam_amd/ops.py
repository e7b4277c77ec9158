"""torch.autograd operators over libnslam.so (HIP, gfx950).  No CPU fallback.

  sample_z        — Renderer.render_batch_ray's sampler (src/utils/Renderer.py:82-170), no grad
  query_points    — NICE.forward + eval_points (decoder.py:168-342, Renderer.py:23-61), fwd+bwd
  composite       — raw2outputs_nerf_color (src/common.py:204-245, occupancy), fwd+bwd
  grid_sample     — F.grid_sample(bilinear, border, align_corners=True) on a channels-last grid
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _lib
from ._lib import check, lib, ptr, stream_ptr

class KernelTimer:
    """Optional live timing of the C-ABI launches with HIP events on the launching stream.

    ops.TIMER = KernelTimer() turns it on (bench.py does, for the timed region only); each entry
    point records an event pair around its launches; summary() synchronises and averages.
    """

    def __init__(self):
        self.events = {}

    def span(self, name):
        return _Span(self, name)

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for name, pairs in self.events.items():
            ms = [a.elapsed_time(b) for a, b in pairs]
            out[name] = {"calls": len(ms), "avg_ms": sum(ms) / max(len(ms), 1), "total_ms": sum(ms)}
        return out


class _Span:
    def __init__(self, timer, name):
        self.timer, self.name = timer, name

    def __enter__(self):
        self.a = torch.cuda.Event(enable_timing=True)
        self.a.record()
        return self

    def __exit__(self, *exc):
        b = torch.cuda.Event(enable_timing=True)
        b.record()
        self.timer.events.setdefault(self.name, []).append((self.a, b))
        return False


class _NoSpan:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


TIMER = None
_NOSPAN = _NoSpan()


def _span(name):
    return TIMER.span(name) if TIMER is not None else _NOSPAN


_DEC_FOR_STAGE = {
    "coarse": ("coarse",),
    "middle": ("middle",),
    "fine": ("middle", "fine"),
    "color": ("middle", "fine", "color"),
}
_DEC_ID = {"coarse": _lib.DEC_COARSE, "middle": _lib.DEC_MIDDLE, "fine": _lib.DEC_FINE, "color": _lib.DEC_COLOR}
_GRID_KEYS = ("grid_coarse", "grid_middle", "grid_fine", "grid_color")


def channels_last(g: torch.Tensor) -> torch.Tensor:
    """[1,C,Z,Y,X] grid as physically [Z][Y][X][C] (no copy when it already is)."""
    if g.dim() != 5 or g.shape[0] != 1 or g.shape[1] != 32:
        raise ValueError(f"feature grid must be [1,32,Z,Y,X], got {tuple(g.shape)}")
    if g.dtype != torch.float32:
        raise ValueError("feature grids are float32")
    if not g.is_contiguous(memory_format=torch.channels_last_3d):
        g = g.contiguous(memory_format=torch.channels_last_3d)
    return g


def _bound_list(b):
    b = b.detach().to("cpu", torch.float64)
    return [float(v) for v in b[:, 0]], [float(v) for v in b[:, 1]]


# ----------------------------------------------------------------------------------------------
# sampler
# ----------------------------------------------------------------------------------------------
_T_CACHE = {}


def _t_tables(device, s0, s1):
    key = (str(device), s0, s1)
    if key not in _T_CACHE:
        ts = torch.linspace(0.0, 1.0, s0).to(device)
        tu = torch.linspace(0.0, 1.0, max(s1, 1)).double().to(device)
        _T_CACHE[key] = (ts, tu)
    return _T_CACHE[key]


def sample_z(rays_o, rays_d, gt_depth, bound, n_strat, n_surf, lindisp=False, gt_max=None, out=None):
    """z_vals [N, n_strat(+n_surf)] float64 (surface samples only when gt_depth is given).

    gt_max: optional device float scalar = max(gt_depth) over the FULL batch (ray sharding).
    out: optional preallocated z tensor of that shape (persistent buffers of a captured loop).
    """
    ro = rays_o.detach().float().contiguous()
    rd = rays_d.detach().float().contiguous()
    n = ro.shape[0]
    s1 = n_surf if gt_depth is not None else 0
    if out is not None:
        if tuple(out.shape) != (n, n_strat + s1) or out.dtype != torch.float64 or not out.is_contiguous():
            raise ValueError("out must be a contiguous float64 [N, S] tensor")
        z = out
    else:
        z = torch.empty(n, n_strat + s1, dtype=torch.float64, device=ro.device)
    if n == 0:
        return z
    gt = gt_depth.detach().float().reshape(-1).contiguous() if gt_depth is not None else None
    ts, tu = _t_tables(ro.device, n_strat, n_surf)
    lo, hi = _bound_list(bound)
    L = lib()
    wsb = L.nslam_workspace_size(0, n)
    ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device=ro.device)
    with _span("sample_rays"):
        gm = gt_max.detach().float().reshape(1).contiguous() if (gt_max is not None and gt is not None) else None
        rc = L.nslam_sample_rays(ptr(ro), ptr(rd), ptr(gt), ptr(gm), n, (ctypes.c_double * 3)(*lo),
                                 (ctypes.c_double * 3)(*hi), ptr(ts), n_strat, ptr(tu), s1, int(bool(lindisp)),
                                 ptr(z), ptr(ws), wsb, stream_ptr(ro.device))
    check(rc, "nslam_sample_rays")
    return z


# ----------------------------------------------------------------------------------------------
# fused point query
# ----------------------------------------------------------------------------------------------
class QueryMeta:
    """Non-tensor configuration of one query call."""

    def __init__(self, stage, decs, packers, dec_bounds, oob_bound, n_params):
        self.stage = stage
        self.decs = decs                # tuple of decoder names used by the stage
        self.packers = packers          # name → DecoderPacker
        self.dec_bounds = dec_bounds    # name → ([lo]*3, [hi]*3) normalisation bound
        self.oob_bound = oob_bound      # ([lo]*3, [hi]*3) or None (= no OOB test)
        self.n_params = n_params        # name → number of parameter tensors


def _fill_cfg(meta, grids, packed, dgrads, need_pts_grad):
    cfg = _lib.NslamQueryCfg()
    cfg.stage = _lib.STAGES[meta.stage]
    cfg.need_pts_grad = int(bool(need_pts_grad))
    if meta.oob_bound is None:
        lo, hi = [-math.inf] * 3, [math.inf] * 3
    else:
        lo, hi = meta.oob_bound
    for k in range(3):
        cfg.bound_lo[k], cfg.bound_hi[k] = lo[k], hi[k]
    for name in meta.decs:
        d = _DEC_ID[name]
        g, gg = grids[d][:2]
        slot = grids[d][2] if len(grids[d]) > 2 else None
        cfg.grid[d].data = g.data_ptr()
        cfg.grid[d].grad = gg.data_ptr() if gg is not None else None
        cfg.grid[d].slot = slot.data_ptr() if slot is not None else None
        cfg.grid[d].dims[0], cfg.grid[d].dims[1], cfg.grid[d].dims[2] = g.shape[2], g.shape[3], g.shape[4]
        blo, bhi = meta.dec_bounds[name]
        for k in range(3):
            cfg.grid[d].lo[k], cfg.grid[d].hi[k] = blo[k], bhi[k]
        cfg.packed[d] = packed[name].data_ptr()
        cfg.dgrad[d] = meta.packers[name].grad_struct(dgrads.get(name))
    # the fine decoder also reads the middle grid (no gradient through it)
    if "fine" in meta.decs and "middle" not in meta.decs:
        raise ValueError("fine stage needs the middle decoder/grid")
    return cfg


class _Query(torch.autograd.Function):
    @staticmethod
    def forward(ctx, meta, pts, g_coarse, g_middle, g_fine, g_color, *params):
        pts = pts.detach().to(torch.float64).contiguous()
        grids_in = (g_coarse, g_middle, g_fine, g_color)
        grids = [channels_last(g.detach()) if g is not None else None for g in grids_in]
        packed, off = {}, 0
        for name in meta.decs:
            n = meta.n_params[name]
            packed[name] = meta.packers[name].pack(params[off:off + n])
            off += n
        raw = torch.empty(pts.shape[0], 4, dtype=torch.float32, device=pts.device)
        cfg = _fill_cfg(meta, [(g, None) if g is not None else (None, None) for g in grids], packed, {}, False)
        saved = tape = None
        if any(ctx.needs_input_grad):  # ReLU masks for the backward (grad mode is off inside forward)
            saved = torch.empty(lib().nslam_query_saved_size(pts.shape[0]), dtype=torch.uint8, device=pts.device)
            cfg.saved_masks = saved.data_ptr()
            if meta.stage == "color":  # colour weight gradients read the activation tape (ABI v9)
                first = 6 + sum(meta.n_params[n] for n in meta.decs[:meta.decs.index("color")])
                if any(ctx.needs_input_grad[first:first + meta.n_params["color"]]):
                    tape = torch.empty(lib().nslam_query_tape_size(pts.shape[0]) // 4, dtype=torch.float32,
                                       device=pts.device)
                    cfg.act_tape = tape.data_ptr()
        query_fwd_launch(cfg, pts, pts.shape[0], raw)
        ctx.meta = meta
        ctx.packed = packed
        ctx.grids = grids
        ctx.saved_masks = saved
        ctx.tape = tape
        ctx.save_for_backward(pts)
        return raw

    @staticmethod
    def backward(ctx, g_raw):
        meta = ctx.meta
        (pts,) = ctx.saved_tensors
        g_raw = g_raw.contiguous().float()
        need = ctx.needs_input_grad
        need_pts = bool(need[1])
        grid_grads = [None] * 4
        pairs = []
        for d in range(4):
            g = ctx.grids[d]
            if g is not None and need[2 + d]:
                grid_grads[d] = torch.zeros_like(g, memory_format=torch.channels_last_3d)
            pairs.append((g, grid_grads[d]) if g is not None else (None, None))
        dgrads, off, pidx = {}, 0, 6
        for name in meta.decs:
            n = meta.n_params[name]
            if any(need[pidx + off + i] for i in range(n)):
                dgrads[name] = torch.zeros(meta.packers[name].n_params, dtype=torch.float32, device=pts.device)
            off += n
        g_pts = torch.empty_like(pts) if need_pts else None
        cfg = _fill_cfg(meta, pairs, ctx.packed, dgrads, need_pts)
        if ctx.saved_masks is not None:
            cfg.saved_masks = ctx.saved_masks.data_ptr()
        if ctx.tape is not None:
            cfg.act_tape = ctx.tape.data_ptr()
        wsb = lib().nslam_query_bwd_workspace_size(ctypes.byref(cfg), pts.shape[0])
        ws = torch.empty(wsb, dtype=torch.uint8, device=pts.device) if wsb else None
        with _span("query_bwd"):
            rc = lib().nslam_query_bwd(ctypes.byref(cfg), ptr(pts), pts.shape[0], ptr(g_raw), ptr(g_pts), ptr(ws),
                                       wsb, stream_ptr(pts.device))
        check(rc, "nslam_query_bwd")
        out = [None, g_pts] + grid_grads
        for name in meta.decs:
            n = meta.n_params[name]
            if name in dgrads:
                out += meta.packers[name].split_grad(dgrads[name])
            else:
                out += [None] * n
        return tuple(out)


def query_points(nice, p, c_grid, stage, oob_bound=None):
    """raw [P,4] for points p [P,3] (float64) — NICE.forward (+ eval_points' OOB rule)."""
    if stage not in _DEC_FOR_STAGE:
        raise ValueError(f"unknown stage {stage!r}")
    decs = _DEC_FOR_STAGE[stage]
    packers, bounds, nparams, params = {}, {}, {}, []
    for name in decs:
        dec = nice.decoder(name)
        packers[name] = dec.packer()
        bounds[name] = _bound_list(dec.bound)
        plist = list(dec.parameters())
        nparams[name] = len(plist)
        params += plist
    meta = QueryMeta(stage, decs, packers, bounds, None if oob_bound is None else _bound_list(oob_bound), nparams)
    grids = []
    for d, key in enumerate(_GRID_KEYS):
        used = (d == _lib.DEC_COARSE and stage == "coarse") or (d == _lib.DEC_MIDDLE and stage != "coarse") or \
               (d == _lib.DEC_FINE and stage in ("fine", "color")) or (d == _lib.DEC_COLOR and stage == "color")
        grids.append(c_grid[key] if used else None)
    p = p.reshape(-1, 3)
    if p.dtype != torch.float64:
        p = p.double()
    return _Query.apply(meta, p, *grids, *params)


# ----------------------------------------------------------------------------------------------
# one decoder alone: MLP.forward / MLP_no_xyz.forward (decoder.py:177-203, 262-274)
# ----------------------------------------------------------------------------------------------
_ZERO_PACKED = {}


class _Stub:
    """Stands in for a decoder the kernel's stage evaluates beside the one asked for (its output is
    discarded): all-zero packed weights, no parameters, no gradient."""

    def __init__(self, nc, device):
        from .packing import xyz_layout
        key = (nc, str(device))
        if key not in _ZERO_PACKED:
            _ZERO_PACKED[key] = torch.zeros(xyz_layout(nc)["total"], dtype=torch.float32, device=device)
        self.packed = _ZERO_PACKED[key]

    def pack(self, params):
        return self.packed

    def grad_struct(self, base):
        return _lib.NslamDecGrad()


class _OneDecoder(torch.autograd.Function):
    """The fine or colour decoder evaluated alone, through the stage that holds it (fine: middle |
    fine, colour: middle | fine | colour) with the other decoders as zero stubs: the fine
    occupancy comes from the forward's deferred-combine mode (raw[...,3] = fine only), the colour
    decoder's rgb from raw[..., :3], and its 4th output row (which NICE.forward overwrites,
    decoder.py:341) from the forward's activation tape h4 (returned as a second output so torch
    forms h4 @ Wo[3] + bo[3]).  Backward: that decoder's share only (nslam_query_bwd_decoder); the
    cotangent torch forms for h4 (the 4th row's Wo[3] g) enters the kernels' Woᵀg as
    nslam_query_cfg.g_h4 (ABI v17), so it reaches the hidden layers, the grid and the points."""

    @staticmethod
    def forward(ctx, meta, name, pts, g_own, g_middle, *params):
        ctx.set_materialize_grads(False)
        pts = pts.detach().to(torch.float64).contiguous()
        n = pts.shape[0]
        own = channels_last(g_own.detach())
        mid = channels_last(g_middle.detach()) if g_middle is not None else own
        d = _DEC_ID[name]
        grids = [None] * 4
        grids[_lib.DEC_MIDDLE] = (mid, None)
        grids[_lib.DEC_FINE] = (own if name == "fine" else mid, None)
        grids[d] = (own, None)
        packed = {k: meta.packers[k].pack(params if k == name else ()) for k in meta.decs}
        cfg = _fill_cfg(meta, grids, packed, {}, False)
        raw = torch.empty(n, 4, dtype=torch.float32, device=pts.device)
        saved = torch.empty(lib().nslam_query_saved_size(n), dtype=torch.uint8, device=pts.device)
        cfg.saved_masks = saved.data_ptr()
        tape = None
        if name == "color":
            tape = torch.empty(lib().nslam_query_tape_size(n) // 4, dtype=torch.float32, device=pts.device)
            cfg.act_tape = tape.data_ptr()
        if n:
            query_fwd_launch(cfg, pts, n, raw, split=True, defer_occ=name == "fine")
        ctx.meta, ctx.name, ctx.grids, ctx.packed = meta, name, grids, packed
        ctx.saved_masks, ctx.tape = saved, tape
        ctx.save_for_backward(pts)
        if name == "fine":
            return raw[:, 3].clone(), None
        # h4 of point i: tape [tile][layer][32 points][32 features], layer 4 (nslam.h act_tape)
        h4 = tape.view(-1, 5, 32, 32)[:, 4].reshape(-1, 32)[:n].clone()
        return raw[:, :3].clone(), h4

    @staticmethod
    def backward(ctx, g_out, g_h4):
        meta, name = ctx.meta, ctx.name
        (pts,) = ctx.saved_tensors
        need = ctx.needs_input_grad
        n = pts.shape[0]
        d = _DEC_ID[name]
        g_raw = torch.zeros(n, 4, dtype=torch.float32, device=pts.device)
        if g_out is not None:
            if name == "fine":
                g_raw[:, 3] = g_out
            else:
                g_raw[:, :3] = g_out
        grids = list(ctx.grids)
        own = grids[d][0]
        g_grid = torch.zeros_like(own, memory_format=torch.channels_last_3d) if need[3] else None
        grids[d] = (own, g_grid)
        dgrad = torch.zeros(meta.packers[name].n_params, dtype=torch.float32, device=pts.device) \
            if any(need[5:]) else None
        g_pts = torch.empty_like(pts) if need[2] else None
        cfg = _fill_cfg(meta, grids, ctx.packed, {name: dgrad} if dgrad is not None else {}, need[2])
        cfg.saved_masks = ctx.saved_masks.data_ptr()
        if ctx.tape is not None:
            cfg.act_tape = ctx.tape.data_ptr()
        if g_h4 is not None:  # d/dh4 of the 4th output row (decoder.py:198-203), [n, 32] float32
            g_h4 = g_h4.detach().to(torch.float32).contiguous()
            cfg.g_h4 = g_h4.data_ptr()
        if n and (g_grid is not None or dgrad is not None or g_pts is not None):
            wsb = lib().nslam_query_bwd_decoder_workspace_size(ctypes.byref(cfg), d, n)
            ws = torch.empty(wsb, dtype=torch.uint8, device=pts.device) if wsb else None
            rc = lib().nslam_query_bwd_decoder(ctypes.byref(cfg), d, 0, ptr(pts), n, ptr(g_raw), ptr(g_pts),
                                               ptr(ws), wsb, stream_ptr(pts.device))
            check(rc, "nslam_query_bwd_decoder")
        elif g_pts is not None:
            g_pts.zero_()
        grads = meta.packers[name].split_grad(dgrad) if dgrad is not None else [None] * meta.n_params[name]
        return (None, None, g_pts, g_grid, None, *grads)


def query_decoder(dec, p, c_grid):
    """One decoder's forward (MLP.forward / MLP_no_xyz.forward): coarse [P], middle [P], fine [P]
    (occupancy, out.squeeze(-1)), colour [P, 4] — the reference module's output for p [P, 3]."""
    name = dec.name
    p = p.reshape(-1, 3)
    if p.dtype != torch.float64:
        p = p.double()
    bl = _bound_list(dec.bound)
    params = list(dec.parameters())
    if name in ("coarse", "middle"):
        meta = QueryMeta(name, (name,), {name: dec.packer()}, {name: bl}, None, {name: len(params)})
        grids = [None] * 4
        grids[_DEC_ID[name]] = c_grid["grid_" + name]
        return _Query.apply(meta, p, *grids, *params)[:, 3]
    stage = name
    decs = _DEC_FOR_STAGE[stage]
    packers = {k: (dec.packer() if k == name else _Stub(2 if k == "fine" else 1, p.device)) for k in decs}
    meta = QueryMeta(stage, decs, packers, {k: bl for k in decs}, None, {k: (len(params) if k == name else 0)
                                                                          for k in decs})
    own = c_grid["grid_" + name]
    out, h4 = _OneDecoder.apply(meta, name, p, own, c_grid.get("grid_middle"), *params)
    if name == "fine":
        return out
    W, b = dec.output_linear.weight, dec.output_linear.bias
    return torch.cat([out, (h4 @ W[3] + b[3])[:, None]], 1)


# ----------------------------------------------------------------------------------------------
# compositing
# ----------------------------------------------------------------------------------------------
class _Composite(torch.autograd.Function):
    @staticmethod
    def forward(ctx, raw, z):
        raw = raw.detach().float().contiguous()
        z = z.detach().double().contiguous()
        n, s = z.shape
        depth = torch.empty(n, dtype=torch.float64, device=raw.device)
        var = torch.empty(n, dtype=torch.float64, device=raw.device)
        color = torch.empty(n, 3, dtype=torch.float32, device=raw.device)
        if n:
            with _span("composite_fwd"):
                rc = lib().nslam_composite_fwd(ptr(raw), ptr(z), n, s, ptr(depth), ptr(var), ptr(color),
                                               stream_ptr(raw.device))
            check(rc, "nslam_composite_fwd")
        ctx.save_for_backward(raw, z)
        return depth, var, color

    @staticmethod
    def backward(ctx, gd, gv, gc):
        raw, z = ctx.saved_tensors
        n, s = z.shape
        g_raw = torch.empty_like(raw)
        if n:
            gd = gd.contiguous().double() if gd is not None else None
            gv = gv.contiguous().double() if gv is not None else None
            gc = gc.contiguous().float() if gc is not None else None
            with _span("composite_bwd"):
                rc = lib().nslam_composite_bwd(ptr(raw), ptr(z), n, s, ptr(gd), ptr(gv), ptr(gc), ptr(g_raw),
                                               stream_ptr(raw.device))
            check(rc, "nslam_composite_bwd")
        return g_raw, None


def composite(raw, z):
    """(depth f64 [N], var f64 [N], color f32 [N,3]) from raw [N,S,4] f32, z [N,S] f64."""
    return _Composite.apply(raw, z)


# ----------------------------------------------------------------------------------------------
# standalone trilinear lookup
# ----------------------------------------------------------------------------------------------
class _GridSample(torch.autograd.Function):
    @staticmethod
    def forward(ctx, grid, coords):
        g = channels_last(grid.detach())
        c = coords.detach().float().reshape(-1, 3).contiguous()
        out = torch.empty(c.shape[0], 32, dtype=torch.float32, device=c.device)
        dims = (ctypes.c_int32 * 3)(g.shape[2], g.shape[3], g.shape[4])
        if c.shape[0]:
            check(lib().nslam_grid_sample_fwd(ptr(g), dims, ptr(c), c.shape[0], ptr(out), stream_ptr(c.device)),
                  "nslam_grid_sample_fwd")
        ctx.save_for_backward(g, c)
        return out

    @staticmethod
    def backward(ctx, gout):
        g, c = ctx.saved_tensors
        gg = torch.zeros_like(g, memory_format=torch.channels_last_3d) if ctx.needs_input_grad[0] else None
        gc = torch.empty_like(c) if ctx.needs_input_grad[1] else None
        dims = (ctypes.c_int32 * 3)(g.shape[2], g.shape[3], g.shape[4])
        if c.shape[0]:
            check(lib().nslam_grid_sample_bwd(ptr(g), dims, ptr(c), c.shape[0], ptr(gout.contiguous().float()),
                                              ptr(gg), ptr(gc), stream_ptr(c.device)), "nslam_grid_sample_bwd")
        return gg, gc


SPLIT_FWD = True  # decoder-parallel forward (nslam_query_fwd_ws); False: one wave runs every decoder
# how nslam_query_fwd_ws spreads the decoders over the chip (nslam_query_cfg.fwd_variant, ABI v18):
# 0 = the library's default, FWD_UNITS / FWD_PC / FWD_PARTS force one (the same values bit for bit)
FWD_DEFAULT, FWD_UNITS, FWD_PC, FWD_PARTS = 0, 1, 2, 3
FWD_VARIANT = FWD_DEFAULT


def query_fwd_launch(cfg, pts, n, raw, split=None, defer_occ=False):
    """nslam_query_fwd_ws (decoder-parallel) or nslam_query_fwd (one fused chain per wave).

    defer_occ: leave raw[...,3] = the fine occupancy and return the middle occupancy [n] float
    (or None when the stage has no split) for render_loss(occ_add=...) to add on read."""
    split = SPLIT_FWD if split is None else split
    wsb = lib().nslam_query_fwd_workspace_size(ctypes.byref(cfg), n) if split else 0
    occ = None
    with _span("query_fwd"):
        if wsb:
            ws = torch.empty(wsb, dtype=torch.uint8, device=raw.device)
            cfg.defer_occ = int(bool(defer_occ))
            cfg.fwd_variant = FWD_VARIANT
            rc = lib().nslam_query_fwd_ws(ctypes.byref(cfg), ptr(pts), n, ptr(raw), ptr(ws), wsb,
                                          stream_ptr(raw.device))
            cfg.defer_occ = 0
            if defer_occ:
                occ = ws[:n * 4].view(torch.float32)
        else:
            rc = lib().nslam_query_fwd(ctypes.byref(cfg), ptr(pts), n, ptr(raw), stream_ptr(raw.device))
    check(rc, "nslam_query_fwd")
    return occ


def grid_sample_fwd(grid, coords, out):
    """nslam_grid_sample_fwd without autograd: out [M,32] = trilinear features of the normalised
    coords [M,3] in a channels-last grid (bench / bulk-query form; grid_sample() is the
    differentiable drop-in)."""
    if not grid.is_contiguous(memory_format=torch.channels_last_3d):
        raise ValueError("grid must be channels-last")
    dims = (ctypes.c_int32 * 3)(grid.shape[2], grid.shape[3], grid.shape[4])
    with _span("grid_fwd"):
        rc = lib().nslam_grid_sample_fwd(ptr(grid), dims, ptr(coords), coords.shape[0], ptr(out),
                                         stream_ptr(coords.device))
    check(rc, "nslam_grid_sample_fwd")


def grid_sample_bwd(grid, coords, gout, ggrid, gcoords=None):
    """nslam_grid_sample_bwd without autograd: ggrid += scatter of gout (atomics); gcoords = d/dcoords."""
    dims = (ctypes.c_int32 * 3)(grid.shape[2], grid.shape[3], grid.shape[4])
    with _span("grid_bwd"):
        rc = lib().nslam_grid_sample_bwd(ptr(grid), dims, ptr(coords), coords.shape[0], ptr(gout), ptr(ggrid),
                                         ptr(gcoords), stream_ptr(coords.device))
    check(rc, "nslam_grid_sample_bwd")


def grid_sample(grid, coords):
    """[M,32] trilinear features of normalised coords [M,3] (x,y,z) — F.grid_sample semantics."""
    return _GridSample.apply(grid, coords)


# ----------------------------------------------------------------------------------------------
# fused mapping / tracking iteration (ABI v4): pixel gather, render loss, ray-form query, Adam
# ----------------------------------------------------------------------------------------------
def gather_rays(frames, pix, n_per, H, W, window, fx, fy, cx, cy, bound=None, draw=None, n_kept=None, out=None):
    """get_samples (src/common.py:92-134) for every frame of a window in one launch, plus the
    inside-mask prefilter (Mapper.py:469-481) when `bound` is given.

    frames: list of (depth [H,W] f32, color [H,W,3] f32, c2w [3|4,4] f32) device tensors, or of
    (depth, color, c2w_out [3|4,4] f32, cam [7] f32): the pose formed in the kernel from the camera
    7-vector (nslam_cam_pose's values) and written to c2w_out's first three rows (ABI v21);
    pix: int64 [len(frames)*n_per] select_uv randint indices into each frame's window
    (h0, h1, w0, w1).  Returns rays_o, rays_d [N,3] f32, gt_depth [N] f32 (0 for dropped rays),
    gt_color [N,3] f32, keep [N] uint8.
    pix=None: draw the pixels on the device (`draw`: PixelDraws, ABI v7); n_kept: optional device
    int64 [1] incremented by the number of kept rays; out: optional preallocated
    (rays_o, rays_d, gt_depth, gt_color, keep) to write into.
    """
    nf = len(frames)
    if nf == 0 or nf > _lib.MAX_FRAMES:
        raise ValueError(f"1..{_lib.MAX_FRAMES} frames, got {nf}")
    if pix is None and draw is None:
        raise ValueError("pix or draw")
    dev = pix.device if pix is not None else draw.counter.device
    arr = (_lib.NslamFrame * nf)()
    keepalive = []
    for f, fr in enumerate(frames):
        d, c, m = fr[:3]
        cam = fr[3] if len(fr) > 3 else None
        d = d.detach().float().contiguous()
        c = c.detach().float().contiguous()
        if cam is None:
            m = m.detach().float().contiguous()
        elif m.dtype != torch.float32 or not m.is_contiguous() or cam.dtype != torch.float32 \
                or not cam.is_contiguous() or cam.numel() != 7:
            raise ValueError("a frame given by its camera: c2w_out contiguous f32 [3|4,4], cam contiguous f32 [7]")
        if tuple(d.shape) != (H, W) or tuple(c.shape) != (H, W, 3) or m.shape[-1] != 4 or m.shape[0] < 3:
            raise ValueError("frame tensors must be depth [H,W], color [H,W,3], c2w [3|4,4]")
        keepalive += [d, c, m]
        arr[f].depth, arr[f].color = ptr(d), ptr(c)
        if cam is None:
            arr[f].c2w = ptr(m)
        else:
            arr[f].cam, arr[f].c2w_out = ptr(cam.detach()), ptr(m)
    if pix is not None:
        pix = pix.to(torch.int64).contiguous()
    n = nf * n_per
    if out is not None:
        ro, rd, gd, gc, keep = out
        want = ((n, 3, torch.float32), (n, 3, torch.float32), (n, torch.float32), (n, 3, torch.float32),
                (n, torch.uint8))
        for t, w in zip(out, want):
            if tuple(t.shape) != tuple(w[:-1]) or t.dtype != w[-1] or not t.is_contiguous():
                raise ValueError("out tensors must match gather_rays' outputs")
    else:
        ro = torch.empty(n, 3, dtype=torch.float32, device=dev)
        rd = torch.empty(n, 3, dtype=torch.float32, device=dev)
        gd = torch.empty(n, dtype=torch.float32, device=dev)
        gc = torch.empty(n, 3, dtype=torch.float32, device=dev)
        keep = torch.empty(n, dtype=torch.uint8, device=dev)
    h0, h1, w0, w1 = window
    if bound is not None:
        lo, hi = _bound_list(bound)
        blo, bhi = (ctypes.c_double * 3)(*lo), (ctypes.c_double * 3)(*hi)
    else:
        blo = bhi = None
    with _span("gather_rays"):
        rc = lib().nslam_gather_rays(arr, nf, n_per, ptr(pix), H, W, h0, h1, w0, w1, fx, fy, cx, cy, blo, bhi,
                                     ptr(ro), ptr(rd), ptr(gd), ptr(gc), ptr(keep),
                                     ctypes.byref(draw.struct) if (pix is None) else None,
                                     ptr(n_kept) if n_kept is not None else None, stream_ptr(dev))
    check(rc, "nslam_gather_rays")
    return ro, rd, gd, gc, keep


class PixelDraws:
    """Device state of in-kernel pixel draws (nslam_draw, ABI v7): a seed and a device draw
    counter the gather kernel advances itself — no host RNG work per (graph-replayed) call.
    Uniform over the window like select_uv's torch.randint (common.py:113-134), but a different
    stream (counter-based splitmix64), so draws do not reproduce torch's sequence.

    Ray sharding (world > 1): every rank passes the same seed; the global batch holds
    n_per * world pixels per frame and this rank gathers slots [rank*n_per, (rank+1)*n_per) of
    each frame.  with_max: the kernel also leaves max(gt_depth) over the kept rays of the WHOLE
    global batch in self.gt_max (each rank re-draws the other ranks' slots) — the sampler's
    batch-global scalar (Renderer.py:107-111,144) without an all-reduce."""

    def __init__(self, seed, device, world=1, rank=0, with_max=False):
        if not (world >= 1 and 0 <= rank < world):
            raise ValueError(f"rank {rank} of world {world}")
        self.counter = torch.zeros(1, dtype=torch.int64, device=device)
        self.ticket = torch.zeros(1, dtype=torch.int32, device=device)
        self.world, self.rank = int(world), int(rank)
        self.gt_max = torch.zeros(1, dtype=torch.float32, device=device) if with_max else None
        self.key = torch.zeros(1, dtype=torch.int32, device=device) if with_max else None
        self.struct = _lib.NslamDraw(int(seed) & (2 ** 64 - 1), ptr(self.counter), ptr(self.ticket), self.world,
                                     self.rank, ptr(self.gt_max), ptr(self.key))


def cam_pose(cam, out):
    """nslam_cam_pose (ABI v8): out [3,4] f32 = get_camera_from_tensor(cam [7]) in one launch."""
    if cam.dtype != torch.float32 or tuple(cam.shape) != (7,) or not cam.is_contiguous():
        raise ValueError("cam_pose: cam must be a contiguous float32 [7]")
    if out.dtype != torch.float32 or tuple(out.shape) != (3, 4) or not out.is_contiguous():
        raise ValueError("cam_pose: out must be a contiguous float32 [3, 4]")
    check(lib().nslam_cam_pose(ptr(cam), ptr(out), stream_ptr(cam.device)), "nslam_cam_pose")
    return out


def cam_grad(cam, c2w, g_pts, z, rd, out):
    """nslam_cam_grad (ABI v8): out [7] f32 = d loss / d cam through pts = t + (R·dir)·z and
    get_camera_from_tensor (Renderer.py:172-174, common.py:137-176), from g_pts [N*S,3] f64,
    z [N,S] f64, rays_d [N,3] f32 and the c2w [3,4] f32 the rays were built with."""
    n, S = z.shape
    for t, dt, shp in ((cam, torch.float32, (7,)), (c2w, torch.float32, (3, 4)), (g_pts, torch.float64, (n * S, 3)),
                       (z, torch.float64, (n, S)), (rd, torch.float32, (n, 3)), (out, torch.float32, (7,))):
        if t.dtype != dt or tuple(t.shape) != shp or not t.is_contiguous():
            raise ValueError(f"cam_grad: expected contiguous {dt} {shp}, got {t.dtype} {tuple(t.shape)}")
    with _span("cam_grad"):
        rc = lib().nslam_cam_grad(ptr(cam), ptr(c2w), ptr(g_pts), ptr(z), ptr(rd), n, S, ptr(out), stream_ptr(cam.device))
    check(rc, "nslam_cam_grad")
    return out


def cam_grad_parts(cam, c2w, g_pts, z, rd, out, ws, ticket):
    """nslam_cam_grad_parts (ABI v15): cam_grad from the per-decoder d/dpts buffers g_pts (list of
    [N*S,3] f64, summed per point in list order inside the kernel) over several workgroups; ws: f64
    [NSLAM_CAM_GRAD_WS_DOUBLES], ticket: int32 [1] zeroed once (both persistent, one per caller)."""
    n, S = z.shape
    for t, dt, shp in ((cam, torch.float32, (7,)), (c2w, torch.float32, (3, 4)), (z, torch.float64, (n, S)),
                       (rd, torch.float32, (n, 3)), (out, torch.float32, (7,)), (ws, torch.float64, (384,)),
                       (ticket, torch.int32, (1,))) + tuple((g, torch.float64, (n * S, 3)) for g in g_pts):
        if t.dtype != dt or tuple(t.shape) != shp or not t.is_contiguous():
            raise ValueError(f"cam_grad_parts: expected contiguous {dt} {shp}, got {t.dtype} {tuple(t.shape)}")
    bufs = (ctypes.c_void_p * len(g_pts))(*[ptr(g) for g in g_pts])
    with _span("cam_grad"):
        rc = lib().nslam_cam_grad_parts(ptr(cam), ptr(c2w), bufs, len(g_pts), ptr(z), ptr(rd), n, S, ptr(out), ptr(ws),
                                        ptr(ticket), stream_ptr(cam.device))
    check(rc, "nslam_cam_grad_parts")
    return out


def cam_grad_step(cam, c2w, g_pts, z, rd, g_cam, ws, ticket, adam, ray_loss, loss_out, best_loss=None, best=None):
    """nslam_cam_grad_step (ABI v23): cam_grad_parts, then in its last workgroup the camera's Adam step in
    place (adam = (exp_avg [7], exp_avg_sq [7], step [1], lr, beta1, beta2, eps)), loss_out = the fixed-order
    sum of ray_loss and, with best_loss / best, the best-pose update — bit-identical to cam_grad_parts +
    FusedAdam.step + loss_sum_best, in one launch."""
    n, S = z.shape
    ex, ex2, stp, lr, b1, b2, eps = adam
    checks = ((cam, torch.float32, (7,)), (c2w, torch.float32, (3, 4)), (z, torch.float64, (n, S)),
              (rd, torch.float32, (n, 3)), (g_cam, torch.float32, (7,)), (ws, torch.float64, (384,)),
              (ticket, torch.int32, (1,)), (ex, torch.float32, (7,)), (ex2, torch.float32, (7,)),
              (stp, torch.float32, (1,)), (ray_loss, torch.float64, (ray_loss.numel(),)),
              (loss_out, torch.float64, ()))
    if best_loss is not None:
        checks += ((best_loss, torch.float64, ()), (best, torch.float32, (7,)))
    for t, dt, shp in checks + tuple((g, torch.float64, (n * S, 3)) for g in g_pts):
        if t.dtype != dt or tuple(t.shape) != shp or not t.is_contiguous():
            raise ValueError(f"cam_grad_step: expected contiguous {dt} {shp}, got {t.dtype} {tuple(t.shape)}")
    tail = _lib.NslamCamTail(ptr(cam), ptr(ex), ptr(ex2), ptr(stp), float(lr), float(b1), float(b2), float(eps),
                             ptr(ray_loss), ray_loss.numel(), ptr(loss_out), ptr(best_loss), ptr(best))
    bufs = (ctypes.c_void_p * len(g_pts))(*[ptr(g) for g in g_pts])
    with _span("cam_grad"):
        rc = lib().nslam_cam_grad_step(ctypes.byref(tail), ptr(c2w), bufs, len(g_pts), ptr(z), ptr(rd), n, S,
                                       ptr(g_cam), ptr(ws), ptr(ticket), stream_ptr(cam.device))
    check(rc, "nslam_cam_grad_step")
    return loss_out


CAM_GRAD_WS_DOUBLES = 32 * 12  # NSLAM_CAM_GRAD_WS_DOUBLES


def cam_vector_batch(c2w, out, copy=None):
    """nslam_cam_vector_batch (ABI v22): out[k] = get_tensor_from_camera(c2w[k]) for c2w [n, 3|4, 4] f32
    (common.camera_tensors' arithmetic, one launch); copy: optional second [n, 7] f32 receiving the same."""
    n = c2w.shape[0]
    if c2w.dtype != torch.float32 or c2w.dim() != 3 or c2w.shape[1] not in (3, 4) or c2w.shape[2] != 4 \
            or not c2w.is_contiguous() or not 1 <= n <= 64:
        raise ValueError("cam_vector_batch: c2w must be a contiguous float32 [n, 3|4, 4], 1 <= n <= 64")
    for t in (out,) if copy is None else (out, copy):
        if t.dtype != torch.float32 or tuple(t.shape) != (n, 7) or not t.is_contiguous():
            raise ValueError("cam_vector_batch: out / copy must be contiguous float32 [n, 7]")
    rc = lib().nslam_cam_vector_batch(ptr(c2w), c2w.shape[1] * 4, n, ptr(out), None if copy is None else ptr(copy),
                                      stream_ptr(c2w.device))
    check(rc, "nslam_cam_vector_batch")
    return out


def cam_pose_batch(cams, c2w):
    """nslam_cam_pose_batch (ABI v19): c2w[k, :3, :4] = get_camera_from_tensor(cams[k]) for cams [n, 7] f32
    and c2w [n, 3 or 4, 4] f32 (both contiguous), one launch."""
    n = cams.shape[0]
    if cams.dtype != torch.float32 or cams.dim() != 2 or cams.shape[1] != 7 or not cams.is_contiguous():
        raise ValueError("cam_pose_batch: cams must be a contiguous float32 [n, 7]")
    if (c2w.dtype != torch.float32 or c2w.dim() != 3 or c2w.shape[0] != n or c2w.shape[1] not in (3, 4)
            or c2w.shape[2] != 4 or not c2w.is_contiguous()):
        raise ValueError("cam_pose_batch: c2w must be a contiguous float32 [n, 3|4, 4]")
    with _span("cam_pose"):
        rc = lib().nslam_cam_pose_batch(ptr(cams), ptr(c2w), c2w.shape[1] * 4, n, stream_ptr(cams.device))
    check(rc, "nslam_cam_pose_batch")
    return c2w


def track_best(loss, best_loss, cam, best):
    """nslam_track_best (ABI v20): if loss < best_loss (float64 device scalars): best_loss = loss, best = cam."""
    if loss.dtype != torch.float64 or best_loss.dtype != torch.float64 or cam.dtype != torch.float32 \
            or best.shape != cam.shape or not (cam.is_contiguous() and best.is_contiguous()):
        raise ValueError("track_best: float64 scalars and two contiguous float32 vectors of one shape")
    check(lib().nslam_track_best(ptr(loss), ptr(best_loss), ptr(cam), ptr(best), cam.numel(), stream_ptr(cam.device)),
          "nslam_track_best")


def loss_sum_best(ray_loss, out, best_loss=None, cam=None, best=None):
    """nslam_loss_sum_best (ABI v21): out (float64 device scalar) = ray_loss.sum() in a fixed order (one
    workgroup: the same value on every call); with best_loss: if out < best_loss, best_loss = out and
    best = cam (nslam_track_best's update, Tracker.py:245-247).  Returns out."""
    if ray_loss.dtype != torch.float64 or out.dtype != torch.float64 or not ray_loss.is_contiguous():
        raise ValueError("loss_sum_best: a contiguous float64 ray_loss and a float64 scalar out")
    if best_loss is not None and (best_loss.dtype != torch.float64 or cam.dtype != torch.float32
                                  or best.shape != cam.shape or not (cam.is_contiguous() and best.is_contiguous())):
        raise ValueError("loss_sum_best: a float64 best_loss and two contiguous float32 vectors of one shape")
    check(lib().nslam_loss_sum_best(ptr(ray_loss), ray_loss.numel(), ptr(out),
                                    ptr(best_loss) if best_loss is not None else None,
                                    ptr(cam) if best_loss is not None else None,
                                    ptr(best) if best_loss is not None else None,
                                    cam.numel() if best_loss is not None else 0, stream_ptr(ray_loss.device)),
          "nslam_loss_sum_best")
    return out


def cam_grad_batch(cams, c2w, ray_begin, n_per, g_pts, z, rd, out, ws, tickets):
    """nslam_cam_grad_batch (ABI v19): out [n, 7] = d loss / d cams [n, 7] of the bundle-adjustment cameras,
    camera k's rays being [ray_begin[k], ray_begin[k] + n_per) of the batch (z [N, S] f64, rd [N, 3] f32,
    g_pts: list of [N*S, 3] f64 d/dpts shares); c2w [n, 3|4, 4] the poses rendered with; ws f64
    [n * 384], tickets int32 [n] zeroed once (persistent per caller)."""
    n = cams.shape[0]
    N, S = z.shape
    for t, dt, shp in ((cams, torch.float32, (n, 7)), (z, torch.float64, (N, S)), (rd, torch.float32, (N, 3)),
                       (out, torch.float32, (n, 7)), (ws, torch.float64, (n * CAM_GRAD_WS_DOUBLES,)),
                       (tickets, torch.int32, (n,))) + tuple((g, torch.float64, (N * S, 3)) for g in g_pts):
        if t.dtype != dt or tuple(t.shape) != shp or not t.is_contiguous():
            raise ValueError(f"cam_grad_batch: expected contiguous {dt} {shp}, got {t.dtype} {tuple(t.shape)}")
    if c2w.dtype != torch.float32 or c2w.dim() != 3 or c2w.shape[0] != n or not c2w.is_contiguous():
        raise ValueError("cam_grad_batch: c2w must be a contiguous float32 [n, 3|4, 4]")
    rb = (ctypes.c_int64 * n)(*[int(r) for r in ray_begin])
    bufs = (ctypes.c_void_p * len(g_pts))(*[ptr(g) for g in g_pts])
    with _span("cam_grad"):
        rc = lib().nslam_cam_grad_batch(ptr(cams), ptr(c2w), c2w.shape[1] * 4, n, rb, int(n_per), bufs, len(g_pts),
                                        ptr(z), ptr(rd), N, S, ptr(out), ptr(ws), ptr(tickets), stream_ptr(cams.device))
    check(rc, "nslam_cam_grad_batch")
    return out


def render_loss(raw, z, gt_depth, gt_color, keep=None, mode="mapper", use_color=True, handle_dynamic=False,
                w_color=0.2, want_grad=True, occ_add=None):
    """Mapper/Tracker rendering loss fused with compositing and its backward (see nslam.h).

    raw [N,S,4] (or [N*S,4]) f32, z [N,S] f64.  Returns (depth f64 [N], var f64 [N],
    color f32 [N,3], ray_loss f64 [N], g_raw f32 like raw or None) where sum(ray_loss) is the loss
    and g_raw = dloss/draw.
    """
    z = z.detach().double().contiguous()
    n, s = z.shape
    dev = z.device
    raw = raw.detach().float().contiguous()
    cfg = _lib.NslamLossCfg(_lib.LOSS_MAPPER if mode == "mapper" else _lib.LOSS_TRACKER, int(bool(use_color)),
                            int(bool(handle_dynamic)), float(w_color), ptr(occ_add) if occ_add is not None else None)
    depth = torch.empty(n, dtype=torch.float64, device=dev)
    var = torch.empty(n, dtype=torch.float64, device=dev)
    color = torch.empty(n, 3, dtype=torch.float32, device=dev)
    ray_loss = torch.empty(n, dtype=torch.float64, device=dev)
    g_raw = torch.empty_like(raw) if want_grad else None
    wsb = lib().nslam_render_loss_workspace_size(ctypes.byref(cfg), n)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev) if wsb else None
    gt_depth = gt_depth.detach().float().contiguous()
    gt_color = gt_color.detach().float().contiguous() if gt_color is not None else None
    keep = keep.contiguous() if keep is not None else None
    if n:
        with _span("render_loss"):
            rc = lib().nslam_render_loss(ctypes.byref(cfg), ptr(raw), ptr(z), n, s, ptr(gt_depth), ptr(gt_color),
                                         ptr(keep), ptr(depth), ptr(var), ptr(color), ptr(ray_loss), ptr(g_raw),
                                         ptr(ws), wsb, stream_ptr(dev))
        check(rc, "nslam_render_loss")
    return depth, var, color, ray_loss, g_raw


def rows_pack(grid_flat, rows, tail, out):
    """nslam_rows_pack: out = [grid_flat.view(-1, 32)[rows], tail] (either part may be None)."""
    n = rows.numel() if rows is not None else 0
    nt = tail.numel() if tail is not None else 0
    with _span("rows_xfer"):
        rc = lib().nslam_rows_pack(ptr(grid_flat) if n else None, ptr(rows) if n else None, n, 32, ptr(tail), nt,
                                   ptr(out), stream_ptr(out.device))
    check(rc, "nslam_rows_pack")


def rows_unpack(buf, rows, grid_flat, tail):
    """nslam_rows_unpack: the inverse of rows_pack."""
    n = rows.numel() if rows is not None else 0
    nt = tail.numel() if tail is not None else 0
    with _span("rows_xfer"):
        rc = lib().nslam_rows_unpack(ptr(buf), ptr(rows) if n else None, n, 32, ptr(grid_flat) if n else None,
                                     ptr(tail), nt, stream_ptr(buf.device))
    check(rc, "nslam_rows_unpack")


class FusedAdam:
    """torch.optim.Adam (betas, eps; no weight decay / amsgrad) stepping every parameter segment
    in one HIP launch (nslam_adam_step).  Construction mirrors torch:

        FusedAdam([{"params": [...], "lr": 0.005}, {"params": [grid], "lr": 0.1, "rows": idx}, ...])

    A group's "rows" (int32 device tensor of voxel indices) restricts a channels-last grid to the
    frustum-selected voxels (Mapper.py:314-333): only those rows are updated, in place, with Adam
    state for them alone.  Parameters whose .grad is None are skipped like torch does (their step
    count does not advance); `grads` may map a parameter to an explicit gradient tensor instead.
    Step counts live on the device, so step() can be captured in a hipGraph.
    """

    def __init__(self, groups, betas=(0.9, 0.999), eps=1e-8):
        self.param_groups = []
        self.betas, self.eps = betas, eps
        self.state = {}
        dev = None
        for g in groups:
            g = dict(g)
            g["params"] = list(g["params"])
            self.param_groups.append(g)
            for p in g["params"]:
                dev = p.device
        self.device = dev
        self._tickets = {}  # one step ticket per parameter subset (subsets may step concurrently)
        self.mirrors = {}

    def set_mirror(self, p, idx, dst):
        """After each update also store dense parameter p into dst at idx ([p.numel(), 2] int32,
        -1 = none): keeps a decoder's MFMA-packed copy current inside the Adam launch."""
        if idx.shape != (p.numel(), 2) or idx.dtype != torch.int32 or not idx.is_contiguous():
            raise ValueError("mirror index must be int32 [numel, 2]")
        self.mirrors[p] = (idx, dst)

    def _st(self, p, rows):
        st = self.state.get(p)
        if st is None:
            if rows is not None:
                n = rows.numel() * 32
                ex, ex2 = (torch.zeros(n, dtype=torch.float32, device=p.device) for _ in range(2))
            else:
                ex, ex2 = torch.zeros_like(p), torch.zeros_like(p)
            st = {"exp_avg": ex, "exp_avg_sq": ex2, "step": torch.zeros(1, dtype=torch.float32, device=p.device)}
            self.state[p] = st
        return st

    def segments(self, grads=None):
        segs = []
        for g in self.param_groups:
            rows = g.get("rows")
            for p in g["params"]:
                gr = grads.get(p) if grads is not None else p.grad
                if gr is None:
                    continue
                st = self._st(p, rows)
                s = _lib.NslamAdamSeg()
                s.param, s.grad = ptr(p.data), ptr(gr)
                s.exp_avg, s.exp_avg_sq, s.step = ptr(st["exp_avg"]), ptr(st["exp_avg_sq"]), ptr(st["step"])
                if rows is not None:
                    # grad: dense like the grid, or compact [n_rows][32] in row-list order (engine
                    # frustum-compacted gradients, ABI v6)
                    compact = gr.dim() == 2
                    if compact and not (gr.is_contiguous() and gr.shape == (rows.numel(), p.shape[1])):
                        raise ValueError("compact grid gradient must be [n_rows, 32] contiguous")
                    if not (p.is_contiguous(memory_format=torch.channels_last_3d) and
                            (compact or gr.is_contiguous(memory_format=torch.channels_last_3d))):
                        raise ValueError("row-masked Adam needs channels-last grid and grad")
                    s.rows, s.n, s.row_len = ptr(rows), rows.numel(), p.shape[1]
                    s.grad_rows = int(compact)
                    if g.get("n_live") is not None:  # ABI v19: rows sized for a capacity, live count on the device
                        s.n_live = ptr(g["n_live"])
                else:  # elementwise over storage: any dense layout shared by param, grad and state
                    dense = p.is_contiguous() or p.is_contiguous(memory_format=torch.channels_last_3d)
                    if not (dense and gr.stride() == p.stride() and st["exp_avg"].stride() == p.stride()):
                        raise ValueError("dense Adam segments need param, grad and state of one dense layout")
                    s.rows, s.n, s.row_len = None, p.numel(), 0
                    mi = self.mirrors.get(p)
                    if mi is not None:
                        s.mirror_idx, s.mirror = ptr(mi[0]), ptr(mi[1])
                s.lr = float(g["lr"])
                segs.append((s, p, gr))
        return segs

    @torch.no_grad()
    def step(self, grads=None, zero_grad=False):
        segs = self.segments(grads)
        if not segs:
            return
        if len(segs) > _lib.ADAM_MAX_SEGS:
            raise ValueError(f"at most {_lib.ADAM_MAX_SEGS} parameter tensors per step (flatten the decoders)")
        arr = (_lib.NslamAdamSeg * len(segs))(*[s for s, _, _ in segs])
        b1, b2 = self.betas
        key = tuple(id(p) for _, p, _ in segs)
        ticket = self._tickets.get(key)
        if ticket is None:
            # a ticket made during capture would come from the graph's private pool with its zero-fill
            # baked into the graph: every subset must step once eagerly first
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("FusedAdam: first step of a parameter subset inside graph capture; "
                                   "run one eager step of it before capturing")
            ticket = self._tickets[key] = torch.zeros(1, dtype=torch.int32, device=self.device)
        with _span("adam"):
            rc = lib().nslam_adam_step(arr, len(segs), b1, b2, self.eps, int(bool(zero_grad)), ptr(ticket),
                                       stream_ptr(self.device))
        check(rc, "nslam_adam_step")

    def group_of(self, p):
        """The parameter group holding p."""
        for g in self.param_groups:
            if any(q is p for q in g["params"]):
                return g
        raise KeyError("not a parameter of this optimiser")

    def state_of(self, p):
        """(exp_avg, exp_avg_sq, step) of p, created on first use (dense, or [n_rows * row_len] for a
        row-masked group, as step() keeps them)."""
        st = self._st(p, self.group_of(p).get("rows"))
        return st["exp_avg"], st["exp_avg_sq"], st["step"]

    @torch.no_grad()
    def step_segments(self, segs, key, zero_grad=False):
        """nslam_adam_step over explicit segments (NslamAdamSeg structs built by the caller — e.g. one
        rank's slices of the parameters, distributed.ShardedAdamExchange), with this optimiser's
        betas / eps and a ticket of its own per `key`.  A parameter's step count must appear in at
        most one segment of the call."""
        if not segs:
            return
        if len(segs) > _lib.ADAM_MAX_SEGS:
            raise ValueError(f"at most {_lib.ADAM_MAX_SEGS} segments per step")
        ticket = self._tickets.get(key)
        if ticket is None:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("FusedAdam: first step of a segment set inside graph capture; run one eager step")
            ticket = self._tickets[key] = torch.zeros(1, dtype=torch.int32, device=self.device)
        arr = (_lib.NslamAdamSeg * len(segs))(*segs)
        b1, b2 = self.betas
        with _span("adam"):
            rc = lib().nslam_adam_step(arr, len(segs), b1, b2, self.eps, int(bool(zero_grad)), ptr(ticket),
                                       stream_ptr(self.device))
        check(rc, "nslam_adam_step")

    def init_state(self):
        """Create every parameter's Adam state now (buffers a hipGraph captured later can hold by address)."""
        for g in self.param_groups:
            for p in g["params"]:
                self._st(p, g.get("rows"))

    @torch.no_grad()
    def reset_state(self):
        """Zero every parameter's Adam state (moments and step count) in place: the optimiser then behaves
        as a freshly built one (Mapper.optimize_map re-creates its Adam per call, Mapper.py:365-389), while
        the state buffers — which captured hipGraphs hold by address — stay where they are."""
        for st in self.state.values():
            st["exp_avg"].zero_()
            st["exp_avg_sq"].zero_()
            st["step"].zero_()

    def prepare(self, grads=None):
        """Create (eagerly, outside any graph capture) the Adam state and the step ticket of the parameter
        subset a step(grads) would update, so the step can be captured in a hipGraph."""
        segs = self.segments(grads)
        key = tuple(id(p) for _, p, _ in segs)
        if segs and key not in self._tickets:
            self._tickets[key] = torch.zeros(1, dtype=torch.int32, device=self.device)

    def zero_grad(self, set_to_none=True):
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is not None:
                    if set_to_none:
                        p.grad = None
                    else:
                        p.grad.zero_()
