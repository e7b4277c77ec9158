"""Fused NICE-SLAM mapping iteration on the HIP kernels, without autograd.

One iteration of Mapper.optimize_map's inner loop (src/Mapper.py:421-519) is

    randint pixels → get_samples + inside-mask     nslam_gather_rays        (1 launch)
    sampler                                         nslam_sample_rays        (2-3 launches)
    pts = o + d·z, grids + decoders → raw          nslam_query_fwd, ray form
    compositing + mapping loss + their backward    nslam_render_loss        (1 launch)
    zero gradients                                  one memset over a flat buffer
    decoders + grids backward                      nslam_query_bwd, ray form
    [ray-sharded: RCCL all-reduce of the gradients]
    Adam over frustum-masked grid rows + decoders  nslam_adam_step          (1 launch)
    re-pack the optimised decoder                   one gather

with every buffer persistent, so the whole iteration can be captured in a hipGraph.  The maths
is the reference's: the inside-mask drops rays by zero loss weight instead of compaction (their
gradients are exactly zero and the sampler's batch max only sees kept rays), and Adam updates
the frustum-selected voxels in place instead of through masked copies (Mapper.py:314-333,
394-401, 511-519) — the same elementwise update.
"""
from __future__ import annotations

import ctypes
import os
import math

import numpy as np
import torch

from . import _lib, ops
from ._lib import check, lib, ptr, stream_ptr
from .common import get_camera_from_tensor

_GRID_OF = {"coarse": "grid_coarse", "middle": "grid_middle", "fine": "grid_fine", "color": "grid_color"}


class FlatDecoder:
    """A decoder's parameters re-bound as views of one flat float32 buffer (named_parameters
    order = the nslam_dec_grad layout) with a trailing zero slot, so packing is one gather into a
    persistent buffer and Adam sees one dense segment.  Parameter identity (and state_dict keys)
    is unchanged."""

    def __init__(self, dec):
        self.dec = dec
        self.packer = dec.packer()
        params = list(dec.parameters())
        n = sum(p.numel() for p in params)
        dev = params[0].device
        flat = torch.zeros(n + 1, dtype=torch.float32, device=dev)
        off = 0
        with torch.no_grad():
            for p in params:
                k = p.numel()
                flat[off:off + k].copy_(p.detach().reshape(-1))
                p.data = flat[off:off + k].view_as(p)
                off += k
        self.flat = flat
        self.param = flat[:n]                       # Adam segment
        self.grad = torch.zeros(n, dtype=torch.float32, device=dev)
        self.packed = torch.empty(self.packer.index.shape[0], dtype=torch.float32, device=dev)
        self.idx = self.packer.device_index(dev)
        # inverse of the packing gather: the (at most two) packed slots of each parameter, so Adam
        # can store an updated parameter straight into the packed copy (FusedAdam.set_mirror)
        idx = self.packer.index
        slots = np.full((n, 2), -1, dtype=np.int32)
        pos = np.nonzero(idx >= 0)[0]
        order = np.argsort(idx[pos], kind="stable")
        src, dst = idx[pos][order], pos[order]
        first = np.ones(src.size, dtype=bool)
        first[1:] = src[1:] != src[:-1]
        slots[src[first], 0] = dst[first]
        slots[src[~first], 1] = dst[~first]
        self.mirror_idx = torch.from_numpy(slots).to(dev)
        self.repack()

    def repack(self):
        torch.index_select(self.flat, 0, self.idx, out=self.packed)


class MappingEngine:
    """Fused mapping iterations over shared grids `c` (dict of [1,32,Z,Y,X] channels-last grids)
    and a NICE decoder stack, for the stage schedule of Mapper.optimize_map."""

    def __init__(self, nice, c, bound, n_strat, n_surf, lindisp=False, w_color=0.2, device="cuda", grid_grads=True,
                 rows=None):
        self.nice, self.c, self.bound = nice, c, bound
        self.n_strat, self.n_surf, self.lindisp, self.w_color = n_strat, n_surf, lindisp, w_color
        self.device = torch.device(device)
        names = [n for n in ("coarse", "middle", "fine", "color") if hasattr(nice, n + "_decoder")]
        self.decs = {n: FlatDecoder(nice.decoder(n)) for n in names}
        self.dec_bounds = {n: ops._bound_list(nice.decoder(n).bound) for n in names}
        self.oob = ops._bound_list(bound)
        self._saved = None  # ReLU masks of the last query_fwd (read by query_bwd)
        self._tape = None   # colour-decoder activation tape of the last query_fwd (ABI v9)
        self.occ_add = None  # middle occupancy of the last deferred-combine query_fwd
        self._draws = None   # (seed, ops.PixelDraws) of in-kernel pixel draws
        self._pre = None     # (key, [buffer set 0, buffer set 1]) ray batches of the prefetch loop
        self._parity = 0     # which set holds this iteration's batch
        self._pre_stream = None
        self._side = []     # side streams of the concurrent decoder backward
        self.concurrent = True
        self.priority = False  # concurrent: run the weight-gradient branch on a high-priority stream
        self.all_side = False  # concurrent: every branch on a side stream (main only forks / joins)
        self.lean_first = False  # concurrent: enqueue the frozen decoders' branches before the weight-gradient one
        # frozen decoders' mask-only backward as one launch (ABI v10) whenever there are several
        # (tracking: 0.199 -> 0.117 ms per iteration; mapping, beside the colour branch's lean chain +
        # k_color_wgrad: 205-208 vs 195-197 M ray-samples/s, profiles/r03_knobs.txt); False = one
        # launch per decoder; "all": every decoder, the colour weight gradients included, in one
        # launch (experiment)
        self.merge_frozen = True
        # ABI v11 split: the colour lean chain alone first, then its weight-gradient reduction beside
        # the frozen decoders' backward (wgrad_side: which of the two forks off).  Measured slower
        # (182 vs 199 M ray-samples/s, profiles/r03_knobs.txt): the lean kernels are latency-bound at
        # the colour chain's 1500 waves (60 us alone vs 76 us for all three decoders together).
        self.split_wgrad = False
        self.wgrad_side = True
        # merged d/dpts summed inside the launch (NSLAM_BWD_SUM_PTS, one workgroup per tile): measured
        # 0.109 vs 0.102 ms per tracking iteration for per-decoder buffers + two adds — kept off
        self.sum_pts = False
        # ABI v14: with per-branch Adam the colour branch may fold the colour decoder's and colour
        # grid's Adam step into the weight-gradient slab reduction (nslam_color_wgrad_adam) — one
        # launch fewer.  Measured 199-203 vs 206-208 M ray-samples/s for the separate Adam launch in
        # the hipGraph'd room0 iteration (the fused reduction takes 16.7 us against 8.8 + 9.7): off.
        self.fuse_adam = os.environ.get("NSLAM_FUSE_ADAM", "0") == "1"
        # the colour grid's Adam in the frozen branch's Adam call (that stream waits for the colour
        # lean chain), off the colour branch's critical path: lean -> weight gradients -> decoder Adam
        self.cgrid_side = os.environ.get("NSLAM_CGRID_SIDE", "1") == "1"
        self._lean_ev = None
        # Cross-iteration pipelining (colour stage, one rank, per-branch Adam; experiment, off: measured
        # 181-185 vs 206-208 M ray-samples/s — the two forward halves side by side take 100 us against
        # the single decoder-parallel launch's 91 us, which the overlap does not win back): the colour
        # branch (lean chain -> weight gradients with the colour decoder's and grid's Adam, ABI v14)
        # stays on its own stream past the end of iteration(), and the next iteration's forward is
        # split (ABI v13 nslam_query_fwd_parts): its middle | fine parts — which read neither the
        # colour grid nor the colour decoder — start as soon as the frozen branch's grid Adam is done,
        # its colour part queues behind the colour branch.  Every iteration still sees the map its predecessor
        # left (the same dependencies as the serial loop).  Callers join() before reading the colour
        # decoder / grid or ending a graph capture.
        self.pipeline = False
        self._col_pending = False
        self._col_stream = None   # the colour branch (+ the next forward's colour part)
        self._hi = None
        for k, v in c.items():
            if not v.is_contiguous(memory_format=torch.channels_last_3d):
                raise ValueError(f"{k} must be channels-last (ops.channels_last)")
        self.grid_grads = grid_grads
        self.set_rows(rows)

    def set_rows(self, rows):
        """Grid-gradient layout.  rows=None: dense gradients (one flat buffer for every grid, so
        zeroing is a single memset).  rows={grid key: int32 voxel rows} (the frustum selection of
        Mapper.py:314-333, the FusedAdam group "rows"): those grids accumulate a COMPACT gradient
        [n_rows][32] in row-list order through a voxel→slot map (ABI v6 nslam_grid.slot); the
        scatter skips every other voxel, whose gradient the reference never forms (it optimises
        the masked vector, Mapper.py:394-401).  Adam then reads the compact rows directly and the
        ray-sharded exchange all-reduces them as they are."""
        c = self.c
        self.rows = dict(rows) if rows else {}
        self.slot = {}
        sizes = {}
        for k, v in c.items():
            sizes[k] = 0 if not self.grid_grads else (self.rows[k].numel() * 32 if k in self.rows else v.numel())
        # one flat gradient buffer: the grids (c order), then the decoders' gradients (colour first, so
        # the colour stage's whole exchange payload — middle/fine/colour rows + colour decoder — is
        # one contiguous span of it: all-reduced in place, distributed.SparseGradExchange)
        dorder = [n for n in ("color", "fine", "middle", "coarse") if n in self.decs]
        gsum = sum(sizes.values())
        self.gall = torch.zeros(gsum + sum(self.decs[n].param.numel() for n in dorder), dtype=torch.float32,
                                device=self.device)
        self.gbuf = self.gall[:gsum]
        off = gsum
        for n in dorder:
            k = self.decs[n].param.numel()
            self.decs[n].grad = self.gall[off:off + k]
            off += k
        self._clean = False  # every gradient the next iteration accumulates into is known zero
        self.ggrad, off = {}, 0
        for k, v in c.items():
            if not self.grid_grads:  # tracking: grids are constants (Tracker.py:138-141)
                continue
            Z, Y, X = v.shape[2:]
            if k in self.rows:
                r = self.rows[k]
                slot = torch.full((Z * Y * X,), -1, dtype=torch.int32, device=self.device)
                slot[r.long()] = torch.arange(r.numel(), dtype=torch.int32, device=self.device)
                self.slot[k] = slot
                self.ggrad[k] = self.gbuf[off:off + sizes[k]].view(-1, 32)
            else:
                self.ggrad[k] = self.gbuf[off:off + sizes[k]].view(1, Z, Y, X, 32).permute(0, 4, 1, 2, 3)
            off += sizes[k]

    # -- query in ray form ---------------------------------------------------------------------
    def _cfg(self, stage, ro, rd, z, grid_grads, dec_grads):
        decs = ops._DEC_FOR_STAGE[stage]
        meta = ops.QueryMeta(stage, decs, {n: self.decs[n].packer for n in decs},
                             {n: self.dec_bounds[n] for n in decs}, self.oob, None)
        pairs = [(None, None, None)] * 4
        for n in decs:
            key = _GRID_OF[n]
            gg = key in grid_grads
            pairs[ops._DEC_ID[n]] = (self.c[key], self.ggrad[key] if gg else None, self.slot.get(key) if gg else None)
        packed = {n: self.decs[n].packed for n in decs}
        dg = {n: self.decs[n].grad for n in decs if n in dec_grads}
        cfg = ops._fill_cfg(meta, pairs, packed, dg, False)
        cfg.rays_o, cfg.rays_d, cfg.z_vals, cfg.n_samples = ptr(ro), ptr(rd), ptr(z), z.shape[1]
        cfg.saved_masks = ptr(self._saved)
        cfg.act_tape = ptr(self._tape)
        return cfg

    def query_fwd(self, stage, ro, rd, z, defer_occ=False, tape=False):
        """raw [N*S, 4]; also saves the ReLU masks the backward of frozen decoders uses.
        defer_occ: raw[...,3] holds the fine occupancy only and self.occ_add the middle one (None
        when the stage has a single occupancy decoder) — render_loss(occ_add=...) adds it.
        tape: also keep the colour decoder's hidden activations for its weight-gradient backward."""
        n = z.numel()
        raw = torch.empty(n, 4, dtype=torch.float32, device=z.device)
        self._saved = torch.empty(lib().nslam_query_saved_size(n), dtype=torch.uint8, device=z.device)
        self._tape = None
        if tape and stage == "color":
            self._tape = torch.empty(lib().nslam_query_tape_size(n) // 4, dtype=torch.float32, device=z.device)
        cfg = self._cfg(stage, ro, rd, z, (), ())
        self.occ_add = ops.query_fwd_launch(cfg, None, n, raw, defer_occ=defer_occ)
        return raw

    def query_bwd(self, stage, ro, rd, z, g_raw, grid_grads, dec_grads, concurrent=None, pts_grad=False,
                  on_branch=None, pts_parts=False):
        """Backward into the engine's gradient buffers.  The decoders write disjoint buffers, so
        each runs as its own launch; with `concurrent` the frozen decoders (mask-only backward,
        atomics-heavy) run on side streams beside the one with weight gradients (MFMA-heavy) —
        parallel branches when captured in a hipGraph.

        pts_grad: also return d loss / d pts [N*S, 3] float64 (tracking, bundle adjustment): every
        decoder writes its share into its own buffer (so the branches stay independent) and the
        shares are summed afterwards.
        on_branch(names): called on each launch's stream right after it, with the decoders it covered
        (the per-branch Adam of the mapping iteration: a grid's rows depend on its branch alone)."""
        n = z.numel()
        self._clean = False
        concurrent = self.concurrent if concurrent is None else concurrent
        cfg = self._cfg(stage, ro, rd, z, grid_grads, dec_grads)
        cfg.need_pts_grad = int(bool(pts_grad))
        decs = sorted(ops._DEC_FOR_STAGE[stage], key=lambda d: d not in dec_grads)  # weight-grad one first
        frozen = [d for d in decs if d not in dec_grads]
        if (self.split_wgrad and concurrent and not pts_grad and list(dec_grads) == ["color"] and frozen
                and self._tape is not None and self._saved is not None and n > 0):
            return self._query_bwd_split(cfg, n, z, g_raw, frozen, on_branch)
        gp = [torch.empty(n, 3, dtype=torch.float64, device=z.device) for _ in decs] if pts_grad else None
        # units of work: (decoder names, stream index); the frozen decoders' mask-only backward is one
        # launch (ABI v10 nslam_query_bwd_decoders) — no fork / join between their streams
        merge = self.merge_frozen
        wgt = [d for d in decs if d in dec_grads]
        if (merge == "all" and self._saved is not None and not pts_grad and wgt == ["color"]
                and self._tape is not None):
            units = [list(decs)]  # every decoder, the colour weight gradients included: one launch
        elif merge and len(frozen) > 1 and self._saved is not None:
            units = [[d] for d in wgt] + [frozen]
        else:
            units = [[d] for d in decs]
        main = torch.cuda.current_stream(z.device)
        streams = [main]
        if concurrent and len(units) > 1:
            while len(self._side) < len(units):
                self._side.append(torch.cuda.Stream(z.device))
            if self.priority:  # the critical (MFMA-heavy) branch gets its waves dispatched first
                if self._hi is None:
                    self._hi = torch.cuda.Stream(z.device, priority=-1)
                streams = [self._hi]
            elif self.all_side:
                streams = [self._side[len(units) - 1]]
            streams += self._side[:len(units) - 1]
        used = [st for st in streams if st is not main]
        cgrid_ev = None  # the colour lean chain's completion, when the colour grid's Adam joins the frozen branch
        summed = False
        with ops._span("query_bwd"):
            for st in used:  # fork: every branch starts from the same point of the main stream
                st.wait_stream(main)
                for t in (ro, rd, z, g_raw, self._saved, self._tape):
                    if t is not None:
                        t.record_stream(st)
            order = list(enumerate(units))
            if concurrent and self.lean_first:
                order = order[1:] + order[:1]
            for i, names in order:
                st = streams[i] if (concurrent and len(units) > 1) else main
                with torch.cuda.stream(st):
                    if len(names) > 1:
                        mask = 0
                        gps = (ctypes.c_void_p * 4)()
                        for name in names:
                            d = ops._DEC_ID[name]
                            mask |= 1 << d
                            if pts_grad:
                                gps[d] = ptr(gp[decs.index(name)])
                        if pts_grad and names == decs and self.sum_pts:
                            # every decoder in this launch: their d/dpts summed in the kernel, in decoder
                            # order (what the loop below would add), into the first buffer
                            mask |= _lib.BWD_SUM_PTS
                            gps[0] = ptr(gp[0])
                            summed = True
                        wsb = 0
                        if "color" in names and "color" in dec_grads:
                            wsb = lib().nslam_query_bwd_decoder_workspace_size(ctypes.byref(cfg), ops._DEC_ID["color"], n)
                        ws = torch.empty(wsb, dtype=torch.uint8, device=z.device) if wsb else None
                        with ops._span("query_bwd." + "+".join(names)):
                            rc = lib().nslam_query_bwd_decoders(ctypes.byref(cfg), mask, None, n, ptr(g_raw), gps,
                                                                ptr(ws), wsb, st.cuda_stream)
                        check(rc, "nslam_query_bwd_decoders")
                    else:
                        name = names[0]
                        d = ops._DEC_ID[name]
                        wsb = lib().nslam_query_bwd_decoder_workspace_size(ctypes.byref(cfg), d, n)
                        ws = torch.empty(wsb, dtype=torch.uint8, device=z.device) if wsb else None
                        tape_bwd = (name == "color" and name in dec_grads and not pts_grad and on_branch is not None
                                    and hasattr(on_branch, "color_wgrad") and self._tape is not None
                                    and self._saved is not None)
                        # the colour grid's Adam beside the weight gradients, in the frozen branch's Adam
                        # (the frozen unit must come after this one: it picks the colour grid's Adam up)
                        cside = (tape_bwd and self.cgrid_side and any(len(u) > 1 for u in units) and concurrent
                                 and not self.lean_first)
                        fused = tape_bwd and (self.fuse_adam or cside)
                        # (the split colour backward is timed as its two kernels: the lean chain and the
                        # weight-gradient reduction have different bounds)
                        with ops._span("query_bwd." + name) if not fused else ops._NOSPAN:
                            if fused:  # lean chain, then weight gradients (+ the colour Adam in the reduction)
                                with ops._span("query_bwd.color_lean"):
                                    rc = lib().nslam_query_bwd_decoders(ctypes.byref(cfg),
                                                                        (1 << d) | _lib.BWD_DEFER_WGRAD, None, n,
                                                                        ptr(g_raw), (ctypes.c_void_p * 4)(), ptr(ws),
                                                                        wsb, st.cuda_stream)
                                check(rc, "nslam_query_bwd_decoders(colour lean)")
                                if cside:
                                    if self._lean_ev is None:  # one persistent event (never destroyed mid-capture)
                                        self._lean_ev = torch.cuda.Event()
                                    self._lean_ev.record(st)
                                    cgrid_ev = self._lean_ev
                                with ops._span("query_bwd.color_wgrad"):
                                    if self.fuse_adam:
                                        on_branch.color_wgrad(cfg, n, ws, wsb, st, grids=not cside)
                                    else:
                                        rc = lib().nslam_color_wgrad(ctypes.byref(cfg), n, ptr(ws), wsb,
                                                                     st.cuda_stream)
                                        check(rc, "nslam_color_wgrad")
                            else:
                                rc = lib().nslam_query_bwd_decoder(ctypes.byref(cfg), d, 0, None, n, ptr(g_raw),
                                                                   ptr(gp[decs.index(name)]) if pts_grad else None,
                                                                   ptr(ws), wsb, st.cuda_stream)
                                check(rc, "nslam_query_bwd_decoder")
                        if fused:
                            if not self.fuse_adam:  # the decoder's Adam (outside the backward's span)
                                on_branch(names, part="decoders")
                            continue
                    if on_branch is not None:
                        if cgrid_ev is not None and len(names) > 1:  # + the colour grid, once its lean chain is done
                            st.wait_event(cgrid_ev)
                            on_branch(list(names) + ["color"], part="grids")
                            cgrid_ev = None
                        else:
                            on_branch(names)
                if pts_grad and st is not main:
                    for name in names:
                        gp[decs.index(name)].record_stream(st)
            for st in used:
                main.wait_stream(st)
        if pts_grad and summed:
            return gp[0]
        if pts_grad and pts_parts:  # the per-decoder shares, for a consumer that sums them itself
            return gp
        if pts_grad:
            out = gp[0]
            for g in gp[1:]:
                out += g
            return out
        return None

    def _query_bwd_split(self, cfg, n, z, g_raw, frozen, on_branch):
        """The mapping iteration's backward with the colour decoder's weight gradients split off
        (ABI v11): the colour lean chain first (its grid gradient and cotangent tape), then its
        weight-gradient reduction (MFMA / LDS bound) on one stream beside the frozen decoders'
        mask-only backward (float-atomic bound) on the other, so the two kinds of work overlap."""
        main = torch.cuda.current_stream(z.device)
        if not self._side:
            self._side.append(torch.cuda.Stream(z.device))
        side = self._side[0]
        dcol = ops._DEC_ID["color"]
        wsb = lib().nslam_query_bwd_decoder_workspace_size(ctypes.byref(cfg), dcol, n)
        ws = torch.empty(wsb, dtype=torch.uint8, device=z.device)
        gps = (ctypes.c_void_p * 4)()
        with ops._span("query_bwd"):
            with ops._span("query_bwd.color_lean"):
                rc = lib().nslam_query_bwd_decoders(ctypes.byref(cfg), (1 << dcol) | _lib.BWD_DEFER_WGRAD, None, n,
                                                    ptr(g_raw), gps, ptr(ws), wsb, main.cuda_stream)
            check(rc, "nslam_query_bwd_decoders(colour lean)")
            side.wait_stream(main)
            for t in (z, g_raw, self._saved, self._tape, ws):
                t.record_stream(side)
            wst, fst = (side, main) if self.wgrad_side else (main, side)
            with torch.cuda.stream(wst):
                with ops._span("query_bwd.color_wgrad"):
                    rc = lib().nslam_color_wgrad(ctypes.byref(cfg), n, ptr(ws), wsb, wst.cuda_stream)
                check(rc, "nslam_color_wgrad")
                if on_branch is not None:
                    on_branch(["color"])
            with torch.cuda.stream(fst):
                mask = 0
                for name in frozen:
                    mask |= 1 << ops._DEC_ID[name]
                with ops._span("query_bwd." + "+".join(frozen)):
                    rc = lib().nslam_query_bwd_decoders(ctypes.byref(cfg), mask, None, n, ptr(g_raw), gps, None, 0,
                                                        fst.cuda_stream)
                check(rc, "nslam_query_bwd_decoders")
                if on_branch is not None:
                    on_branch(frozen)
            main.wait_stream(side)
        return None

    # -- cross-iteration pipelining (self.pipeline) ------------------------------------------------
    def join(self):
        """Make the current stream wait for a pipelined colour branch still in flight (call before
        reading the colour decoder / colour grid, or before ending a graph capture)."""
        if self._col_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._col_stream)
        self._col_pending = False

    def _pipe_streams(self):
        if self._col_stream is None:
            self._col_stream = torch.cuda.Stream(self.device)
        return self._col_stream

    def _query_fwd_pipelined(self, ro, rd, z):
        """Colour-stage forward as two launches: middle | fine on the current stream, colour on the
        colour stream (behind the previous iteration's colour branch); returns raw (occupancy of the
        middle decoder deferred into self.occ_add, as query_fwd(defer_occ=True))."""
        main = torch.cuda.current_stream(self.device)
        sc = self._pipe_streams()
        n = z.numel()
        raw = torch.empty(n, 4, dtype=torch.float32, device=z.device)
        self._saved = torch.empty(lib().nslam_query_saved_size(n), dtype=torch.uint8, device=z.device)
        self._tape = torch.empty(lib().nslam_query_tape_size(n) // 4, dtype=torch.float32, device=z.device)
        cfg = self._cfg("color", ro, rd, z, (), ())
        cfg.defer_occ = 1
        wsb = lib().nslam_query_fwd_workspace_size(ctypes.byref(cfg), n)
        ws = torch.empty(wsb, dtype=torch.uint8, device=z.device)
        # fork BEFORE the middle | fine launch: the colour half needs the rays and the buffers just
        # allocated on main, and (in stream order on sc) the previous iteration's colour branch
        sc.wait_stream(main)
        with ops._span("query_fwd.middle+fine"):
            rc = lib().nslam_query_fwd_parts(ctypes.byref(cfg), None, n, ptr(raw), ptr(ws), wsb, 3, main.cuda_stream)
        check(rc, "nslam_query_fwd_parts(middle | fine)")
        with torch.cuda.stream(sc):
            with ops._span("query_fwd.color"):
                rc = lib().nslam_query_fwd_parts(ctypes.byref(cfg), None, n, ptr(raw), ptr(ws), wsb, 4,
                                                 sc.cuda_stream)
        check(rc, "nslam_query_fwd_parts(colour)")
        main.wait_stream(sc)
        self.occ_add = ws[:n * 4].view(torch.float32)
        return raw

    def _query_bwd_pipelined(self, ro, rd, z, g_raw, keys, frozen, on_branch):
        """The colour stage's backward with per-branch Adam: the colour stream runs the colour lean
        chain, then the weight gradients with the colour decoder's and colour grid's Adam in the
        reduction (ABI v14), and is NOT joined into the current stream (the next iteration's colour
        forward queues behind it); the current stream runs the frozen decoders' merged mask-only
        launch and the middle / fine grids' Adam.  So the next forward's middle | fine half (which
        reads neither the colour grid nor the colour decoder) does not wait for the colour branch.
        (Stream topology chosen for hipGraph capture on this stack: a stream forked off the colour
        stream and joined back into it crashes hipStreamEndCapture, tools/probes/capture_topology.py
        pattern t3.)"""
        main = torch.cuda.current_stream(self.device)
        sc = self._pipe_streams()
        n = z.numel()
        cfg = self._cfg("color", ro, rd, z, keys, ("color",))
        cfg.need_pts_grad = 0
        self._clean = False
        dcol = ops._DEC_ID["color"]
        # the colour workspace is allocated on the current stream (inside a graph capture the caching
        # allocator serves the capturing stream's pool)
        wsb = lib().nslam_query_bwd_decoder_workspace_size(ctypes.byref(cfg), dcol, n)
        ws = torch.empty(wsb, dtype=torch.uint8, device=z.device)
        mask = 0
        for name in frozen:
            mask |= 1 << ops._DEC_ID[name]
        with ops._span("query_bwd"):
            sc.wait_stream(main)
            for t in (ro, rd, z, g_raw, self._saved, self._tape, ws):
                t.record_stream(sc)
            with torch.cuda.stream(sc):
                with ops._span("query_bwd.color"):
                    rc = lib().nslam_query_bwd_decoders(ctypes.byref(cfg), (1 << dcol) | _lib.BWD_DEFER_WGRAD, None, n,
                                                        ptr(g_raw), (ctypes.c_void_p * 4)(), ptr(ws), wsb,
                                                        sc.cuda_stream)
                    check(rc, "nslam_query_bwd_decoders(colour lean)")
                    on_branch.color_wgrad(cfg, n, ws, wsb, sc)  # (+ the colour decoder's and grid's Adam)
            with ops._span("query_bwd." + "+".join(frozen)):
                rc = lib().nslam_query_bwd_decoders(ctypes.byref(cfg), mask, None, n, ptr(g_raw),
                                                    (ctypes.c_void_p * 4)(), None, 0, main.cuda_stream)
            check(rc, "nslam_query_bwd_decoders")
            on_branch(frozen)
            self._col_pending = True  # the next prefetch reuses this batch's rays: it waits for sc

    # -- one iteration ---------------------------------------------------------------------------
    def grads_for(self, stage, trainable_decoders):
        """(grid keys, decoder names) that receive gradients in `stage` (Mapper.py:335-341)."""
        decs = ops._DEC_FOR_STAGE[stage]
        keys = tuple(_GRID_OF[n] for n in decs)
        return keys, tuple(n for n in decs if n in trainable_decoders)

    def adam_grads(self, stage, trainable_decoders):
        keys, dnames = self.grads_for(stage, trainable_decoders)
        g = {self.c[k]: self.ggrad[k] for k in keys}
        g.update({self.decs[n].param: self.decs[n].grad for n in dnames})
        return g

    def iteration(self, stage, frames, pix, n_per, hw, intrinsics, optimizer, trainable_decoders=("color",),
                  gt_max=None, allreduce=None, use_gt_in_sampler=True, exchange=None, n_kept=None, seed=0,
                  world=1, rank=0, prefetch=False):
        """One mapping iteration; returns (ray_loss f64 [N], keep uint8 [N]) as device tensors.

        frames: [(depth, color, c2w)] of the window; pix: int64 [len(frames)*n_per] randint
        indices over the full image, or None: drawn in the gather kernel (ops.PixelDraws keyed by
        `seed`, advanced on the device — no host RNG work per hipGraph replay; with world > 1 every
        rank passes the same seed, gathers its slice of a global batch of n_per*world pixels per
        frame and gets the global batch's max(gt_depth) from the gather kernel — no collective
        before the sampler); hw = (H, W);
        intrinsics = (fx, fy, cx, cy); n_kept: optional device int64 [1] += kept rays.
        gt_max: callable(gt_depth) → device scalar for a ray-sharded job (all-reduced max);
        allreduce: callable(list of grads) run before Adam (ray sharding, dense);
        exchange: callable(grid keys, decoder names) run before Adam instead — the frustum-compacted
        exchange (distributed.SparseGradExchange).
        prefetch (device draws only): the pixel gather and sampler of the NEXT iteration run on a side
        stream while this one renders and back-propagates — they depend only on the frames and the
        device draw counter, not on the map.  Batches alternate between two persistent buffer sets
        (self._parity), so a hipGraph of an even and one of an odd iteration replay alternately
        with no copies.  Each call still draws, samples, renders and updates one batch; the first
        call draws its own batch first.  The prefetched batch belongs to the frames of the call that
        drew it: a call with other frames (another keyframe window, or poses changed in place, e.g.
        by bundle adjustment — tracked by the tensors' identity and version counters) discards it
        and draws its own batch.  With prefetch the returned `keep` is a persistent buffer, valid
        until the next iteration() call (which overwrites it): clone it to keep it longer.
        """
        H, W = hw
        fx, fy, cx, cy = intrinsics
        draw = None
        if pix is None:
            key = (seed, world, rank)
            if self._draws is None or self._draws[0] != key:
                self._draws = (key, ops.PixelDraws(seed, self.device, world, rank, with_max=world > 1))
            draw = self._draws[1]

        def rays(out=None):  # pixels → rays + inside mask, then the sampler (Mapper.py:457-484, Renderer.py:82-174)
            ro, rd, gd, gc, keep = ops.gather_rays(frames, pix, n_per, H, W, (0, H, 0, W), fx, fy, cx, cy,
                                                   self.bound, draw=draw, n_kept=n_kept,
                                                   out=None if out is None else out[:5])
            gsamp = gd if (use_gt_in_sampler and stage != "coarse") else None
            if gsamp is None:
                gm = None
            elif draw is not None and draw.gt_max is not None:  # global batch max from the gather kernel
                gm = draw.gt_max
            else:
                gm = gt_max(gd) if gt_max is not None else None
            z = ops.sample_z(ro, rd, gsamp, self.bound, self.n_strat, self.n_surf, self.lindisp, gt_max=gm,
                             out=None if out is None else out[5])
            return [ro, rd, gd, gc, keep, z]

        prefetch = prefetch and pix is None
        side = None
        if prefetch:
            # the frames' identity and version counters: a prefetched batch is only valid for the very
            # frames (images and poses, unmodified) it was gathered from
            fkey = tuple((t.data_ptr(), t._version) for f in frames for t in f)
            pkey = (stage, fkey, n_per, hw, use_gt_in_sampler, seed, world, rank)
            if self._pre is None or self._pre[0] != pkey:
                first = rays()  # first call: this iteration's batch (set 0), then a same-shaped set 1
                self._pre = (pkey, [first, [torch.empty_like(t) for t in first]])
                self._parity = 0
            cur, nxt = self._pre[1][self._parity], self._pre[1][1 - self._parity]
            self._parity ^= 1
            main = torch.cuda.current_stream(self.device)
            if self._pre_stream is None:
                self._pre_stream = torch.cuda.Stream(self.device)
            side = self._pre_stream
            side.wait_stream(main)  # the previous iteration's backward has released `nxt`
            if self._col_pending and self._col_stream is not None:
                side.wait_stream(self._col_stream)  # (a pipelined colour lean chain reads `nxt` too)
            with torch.cuda.stream(side):
                rays(out=nxt)  # the next iteration's batch, beside this iteration's render + backward
            ro, rd, gd, gc, keep, z = cur
        else:
            ro, rd, gd, gc, keep, z = rays()
        keys, dnames = self.grads_for(stage, trainable_decoders)
        mirror = hasattr(optimizer, "set_mirror")
        pipe = (self.pipeline and stage == "color" and tuple(dnames) == ("color",)
                and exchange is None and allreduce is None and mirror and hasattr(optimizer, "color_wgrad_step"))
        if not pipe:
            self.join()  # a pipelined predecessor's colour branch must finish before a serial iteration
        if pipe:
            raw = self._query_fwd_pipelined(ro, rd, z)
        else:
            raw = self.query_fwd(stage, ro, rd, z, defer_occ=True, tape="color" in dnames)
        _, _, _, ray_loss, g_raw = ops.render_loss(raw, z, gd, gc, keep, mode="mapper", use_color=stage == "color",
                                                   w_color=self.w_color, occ_add=self.occ_add)
        if not self._clean:
            self.join()  # (a pipelined colour branch may still be writing the decoder gradient)
            self.gall.zero_()  # grid and decoder gradients: one memset
        # Adam resets every gradient entry it reads.  With compact gradients for every grid of the
        # stage that is every entry the backward wrote, so the next iteration needs no memsets.
        clean = all(k in self.rows for k in keys)
        if mirror:  # Adam stores updated decoder parameters straight into their packed copies
            for n in dnames:
                d = self.decs[n]
                if d.param not in optimizer.mirrors:
                    optimizer.set_mirror(d.param, d.mirror_idx, d.packed)
        grads = self.adam_grads(stage, trainable_decoders)
        on_branch = None
        if exchange is None and allreduce is None and mirror:
            # one rank: each decoder branch updates its own grid's rows (+ the trainable decoder's
            # parameters, after its slab reduction) on its own stream — the update of a grid needs
            # that branch's gradients alone, so no branch waits for the others before its Adam
            def on_branch(names, part=None):  # the decoders of one launch: one Adam call for their grids
                sub = {}                         # (part "grids" / "decoders": only those)
                for name in names:
                    if _GRID_OF[name] in keys and part != "decoders":
                        sub[self.c[_GRID_OF[name]]] = grads[self.c[_GRID_OF[name]]]
                    if name in dnames and part != "grids":
                        sub[self.decs[name].param] = grads[self.decs[name].param]
                if sub:
                    optimizer.step(grads=sub, zero_grad=clean)

            if hasattr(optimizer, "color_wgrad_step"):
                def color_wgrad(cfg, n, ws, wsb, st, grids=True):  # weight gradients + the colour Adam, one reduction
                    p = self.decs["color"].param
                    extra = {self.c[k]: grads[self.c[k]] for k in ("grid_color",) if k in keys and grids}
                    optimizer.color_wgrad_step(cfg, n, ws, wsb, p, grads[p], extra=extra, zero_grad=clean, stream=st)

                on_branch.color_wgrad = color_wgrad
        if pipe:
            self._query_bwd_pipelined(ro, rd, z, g_raw, keys, [d for d in ops._DEC_FOR_STAGE[stage] if d != "color"],
                                      on_branch)
        else:
            self.query_bwd(stage, ro, rd, z, g_raw, keys, dnames, on_branch=on_branch)
        if exchange is not None:  # frustum-compacted all-reduce (distributed.SparseGradExchange)
            exchange(keys, dnames)
        elif allreduce is not None:  # the grid gradients as one flat buffer, plus the decoder gradients
            allreduce([self.gbuf] + [self.decs[n].grad for n in dnames])
        if side is not None:  # join: the next call reads the prefetched set
            main.wait_stream(side)
        if on_branch is None:
            optimizer.step(grads=grads, zero_grad=clean)
        self._clean = clean
        if not mirror:
            for n in dnames:
                self.decs[n].repack()
        return ray_loss, keep


def camera_dirs(pix, n_per, n_frames, window, intrinsics, device):
    """Camera-frame ray directions of select_uv pixel draws (src/common.py:80-84, 113-134):
    dirs = ((i-cx)/fx, -(j-cy)/fy, -1) for window index k -> (j, i) = (h0 + k // ww, w0 + k % ww)."""
    h0, h1, w0, w1 = window
    fx, fy, cx, cy = intrinsics
    ww = w1 - w0
    i = (pix % ww + w0).to(torch.float32)
    j = (pix // ww + h0).to(torch.float32)
    d = torch.stack([(i - cx) / fx, -(j - cy) / fy, -torch.ones_like(i)], -1)
    return d.view(n_frames, n_per, 3)


def c2w_grads(g_pts, z, dirs):
    """d loss / d c2w[:3, :4] per frame from d loss / d pts, through pts = o + d·z
    (Renderer.py:172-174), rays_o = t and rays_d = R·dir (common.py:80-89):
    g_t = sum_{r,s} g_pts, g_R = sum_r (sum_s z g_pts) dirᵀ.  dirs [F, n, 3] → [F, 3, 4]."""
    F, n = dirs.shape[:2]
    gp = g_pts.view(F, n, -1, 3)
    g_ro = gp.sum(2).float()
    g_rd = (gp * z.view(F, n, -1, 1)).sum(2).float()
    g_R = torch.einsum("fnm,fnk->fmk", g_rd, dirs)
    return torch.cat([g_R, g_ro.sum(1)[..., None]], 2)


class TrackingEngine:
    """Tracker.optimize_cam_in_batch (src/Tracker.py:71-128) on the HIP kernels, without host
    synchronisation: one camera iteration is

        c2w = get_camera_from_tensor(cam)              (autograd on the 7-vector only)
        pixels → rays + inside mask                    nslam_gather_rays
        sampler, decoders (ray form, ReLU masks saved) nslam_sample_rays, nslam_query_fwd_ws
        compositing + tracker loss + their backward    nslam_render_loss (mode TRACKER, median)
        d loss / d pts, frozen decoders                nslam_query_bwd_decoder (mask-only, 3 branches)
        pts → rays → c2w → cam                         nslam_cam_grad (closed form, include/nslam.h)
        Adam on the camera                             ops.FusedAdam (device step count)

    so `iters` iterations can be captured in one hipGraph.  Grids and decoders are constants
    (Tracker.py:138-141): no grid or weight gradients are formed.  As in the reference, dropped
    rays (inside mask) carry no loss and the handle_dynamic median is over kept rays only.
    """

    def __init__(self, nice, c, bound, n_strat, n_surf, hw, intrinsics, ignore_edge=(20, 20), w_color=0.5,
                 handle_dynamic=True, use_color=True, device="cuda"):
        self.eng = MappingEngine(nice, c, bound, n_strat, n_surf, device=device, grid_grads=False)
        self.bound, self.n_strat, self.n_surf = bound, n_strat, n_surf
        self.H, self.W = hw
        self.intr = intrinsics
        he, we = ignore_edge
        self.window = (he, self.H - he, we, self.W - we)
        self.w_color, self.handle_dynamic, self.use_color = w_color, handle_dynamic, use_color
        self.device = torch.device(device)
        self._c2w = None
        # ABI v15 nslam_cam_grad_parts: the frozen decoders' d/dpts buffers summed inside a
        # multi-workgroup camera-gradient kernel (no torch adds, no single-workgroup reduction)
        self.cam_parts = True
        self._cam_ws = self._cam_ticket = None

    def n_window(self):
        h0, h1, w0, w1 = self.window
        return (h1 - h0) * (w1 - w0)

    def iteration(self, cam, depth, color, pix, optimizer):
        """One camera iteration on frame (depth [H,W], color [H,W,3]) with pixel draws `pix`
        (int64 [n], select_uv indices into the edge-cropped window).  cam: [7] leaf tensor whose
        .grad the optimizer reads.  Returns the loss (device f64 scalar) of the pose BEFORE the step."""
        fx, fy, cx, cy = self.intr
        n = pix.numel()
        if self._c2w is None:
            self._c2w = torch.empty(3, 4, dtype=torch.float32, device=cam.device)
        c2w = ops.cam_pose(cam.detach(), self._c2w)  # get_camera_from_tensor in one launch
        ro, rd, gd, gc, keep = ops.gather_rays([(depth, color, c2w)], pix, n, self.H, self.W, self.window,
                                               fx, fy, cx, cy, self.bound)
        z = ops.sample_z(ro, rd, gd, self.bound, self.n_strat, self.n_surf)
        # the fine + middle occupancy sum is formed by the loss kernel as it reads raw (no combine pass)
        raw = self.eng.query_fwd("color", ro, rd, z, defer_occ=True)
        _, _, _, ray_loss, g_raw = ops.render_loss(raw, z, gd, gc, keep, mode="tracker", use_color=self.use_color,
                                                   handle_dynamic=self.handle_dynamic, w_color=self.w_color,
                                                   occ_add=self.eng.occ_add)
        if cam.grad is None:
            cam.grad = torch.empty_like(cam)
        if self.cam_parts:  # the decoders' d/dpts shares summed inside the multi-workgroup cam_grad (ABI v15)
            if self._cam_ws is None:
                self._cam_ws = torch.zeros(384, dtype=torch.float64, device=cam.device)
                self._cam_ticket = torch.zeros(1, dtype=torch.int32, device=cam.device)
            gps = self.eng.query_bwd("color", ro, rd, z, g_raw, (), (), pts_grad=True, pts_parts=True)
            if torch.is_tensor(gps):
                gps = [gps]
            ops.cam_grad_parts(cam.detach(), c2w, gps, z, rd, cam.grad, self._cam_ws, self._cam_ticket)
        else:
            g_pts = self.eng.query_bwd("color", ro, rd, z, g_raw, (), (), pts_grad=True)
            # the whole pts → rays → c2w → 7-vector chain in one launch
            ops.cam_grad(cam.detach(), c2w, g_pts, z, rd, cam.grad)
        optimizer.step()
        return ray_loss.sum()


def frustum_rows(mask_xyz: torch.Tensor) -> torch.Tensor:
    """int32 voxel rows (z*Y*X + y*X + x, channels-last) of a get_mask_from_c2w mask [X, Y, Z]."""
    m = mask_xyz.permute(2, 1, 0).reshape(-1)
    return torch.nonzero(m).reshape(-1).to(torch.int32)
