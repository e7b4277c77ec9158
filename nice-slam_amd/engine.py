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
import math
import os
import weakref

import numpy as np
import torch

from . import _lib, ops
from ._lib import check, lib, ptr, stream_ptr
from .common import get_camera_from_tensor

_GRID_OF = {"coarse": "grid_coarse", "middle": "grid_middle", "fine": "grid_fine", "color": "grid_color"}


def _env_choice(name, default, allowed):
    """An engine topology knob from the environment, checked against its allowed values (a typo raises
    instead of silently selecting another stream topology)."""
    v = os.environ.get(name, default)
    if v not in allowed:
        raise ValueError(f"{name}={v!r}: expected one of {sorted(allowed)}")
    return v


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
        # concurrent backward: enqueue the colour weight-gradient branch before the grid-gradient one
        # (its workgroups are dispatched first and hold one slot per CU; the lean launch fills the rest)
        self.wgrad_first = _env_choice("NSLAM_WGRAD_FIRST", "1", ("0", "1")) == "1"
        # every mask-only decoder backward as ONE launch (ABI v10); False: one nslam_query_bwd_decoder
        # launch per decoder (the library then runs a colour tape backward's two kernels in sequence)
        self.merge = True
        self._lean_ev = None
        # where the ray prefetch of the next iteration forks off the main stream: "start" (beside the
        # forward) or "after_fwd" (beside the loss and the backward: the forward's waves then have every
        # wave slot of the chip; a prefetch sampler wave resident on a SIMD leaves room for only two of
        # the forward's three)
        self.prefetch_at = _env_choice("NSLAM_PREFETCH_AT", "start", ("start", "after_fwd"))
        # the ray prefetch's stream: the backward's first side stream ("lean", default: one side queue
        # fewer in a captured iteration) or its own ("own"); and one Adam call for the whole update on that
        # stream once both backward branches are done (NSLAM_ADAM_MERGE=1, default) instead of one per
        # branch (0).  A/B, round 5: 0.2177 / 0.2150 / 0.2129 ms per room0 iteration (own, lean, lean +
        # merged Adam; medians of 3 alternating rounds, profiles/r05_experiments/ab_defaults.txt)
        self.prefetch_stream = _env_choice("NSLAM_PREFETCH_STREAM", "lean", ("lean", "own"))
        self.adam_merge = _env_choice("NSLAM_ADAM_MERGE", "1", ("0", "1")) == "1"
        # where the merged Adam runs: after the mask-only launch on its side stream ("side") or on the
        # main stream after the join ("main", experiment)
        self.adam_on = _env_choice("NSLAM_ADAM_ON", "side", ("side", "main"))
        self._wg_ev = None
        for k, v in c.items():
            if not v.is_contiguous(memory_format=torch.channels_last_3d):
                raise ValueError(f"{k} must be channels-last (ops.channels_last)")
        self.grid_grads = grid_grads
        self.layout_gen = 0  # bumped by set_rows: consumers holding views of the buffers re-check it
        self.pad_rows = 1
        self.set_rows(rows)

    def set_rows(self, rows, pad_rows=None):
        """Grid-gradient layout.  rows=None: dense gradients (one flat buffer for every grid, so
        zeroing is a single memset).  rows={grid key: int32 voxel rows} (the frustum selection of
        Mapper.py:314-333, the FusedAdam group "rows"): those grids accumulate a COMPACT gradient
        [n_rows][32] in row-list order through a voxel→slot map (ABI v6 nslam_grid.slot); the
        scatter skips every other voxel, whose gradient the reference never forms (it optimises
        the masked vector, Mapper.py:394-401).  Adam then reads the compact rows directly and the
        ray-sharded exchange sums them as they are.
        pad_rows: every compact grid's rows and every decoder's gradient are padded (with entries
        nothing writes) to a multiple of pad_rows rows / elements, so a stage's gradient span splits
        into equal whole-row shards (distributed.ShardedAdamExchange: pad_rows = world size); None keeps
        the current padding.  Every call reallocates the gradient buffers and bumps self.layout_gen: an
        optimiser's compact Adam state and an exchange built for the old rows are invalid afterwards
        (the exchanges raise; rebuild both for the new rows)."""
        c = self.c
        pad = max(1, int(self.pad_rows if pad_rows is None else pad_rows))
        self.layout_gen += 1
        rup = lambda n: -(-n // pad) * pad  # noqa: E731
        drup = lambda n: -(-n // (32 * pad)) * 32 * pad  # noqa: E731  (decoders: whole rows per shard too)
        self.rows = dict(rows) if rows else {}
        self.pad_rows = pad
        self.slot = {}
        sizes = {}
        for k, v in c.items():
            n = self.rows[k].numel() if k in self.rows else v.numel() // 32  # rows (voxels)
            sizes[k] = 0 if not self.grid_grads else rup(n) * 32
        # one flat gradient buffer: the grids (c order), then the decoders' gradients (colour first, so
        # the colour stage's whole exchange payload — middle/fine/colour rows + colour decoder — is
        # one contiguous span of it: all-reduced in place, distributed.SparseGradExchange)
        dorder = [n for n in ("color", "fine", "middle", "coarse") if n in self.decs]
        gsum = sum(sizes.values())
        self.gall = torch.zeros(gsum + sum(drup(self.decs[n].param.numel()) for n in dorder), dtype=torch.float32,
                                device=self.device)
        self.gbuf = self.gall[:gsum]
        off = gsum
        self.dgrad_pad = {}  # decoder -> its gradient with the padding
        for n in dorder:
            k = self.decs[n].param.numel()
            self.decs[n].grad = self.gall[off:off + k]
            self.dgrad_pad[n] = self.gall[off:off + drup(k)]
            off += drup(k)
        self._clean = False  # every gradient the next iteration accumulates into is known zero
        self.ggrad, self.ggrad_pad, off = {}, {}, 0  # ggrad_pad: flat, with the padding
        for k, v in c.items():
            if not self.grid_grads:  # tracking: grids are constants (Tracker.py:138-141)
                continue
            Z, Y, X = v.shape[2:]
            if k in self.rows:
                r = self.rows[k]
                slot = torch.full((Z * Y * X,), -1, dtype=torch.int32, device=self.device)
                slot[r.long()] = torch.arange(r.numel(), dtype=torch.int32, device=self.device)
                self.slot[k] = slot
                self.ggrad[k] = self.gbuf[off:off + r.numel() * 32].view(-1, 32)
            else:
                self.ggrad[k] = self.gbuf[off:off + v.numel()].view(1, Z, Y, X, 32).permute(0, 4, 1, 2, 3)
            self.ggrad_pad[k] = self.gbuf[off:off + sizes[k]]
            off += sizes[k]

    def bind_masks(self, masks):
        """Per-call frustum selection on the device, without a host read-back and without moving any
        buffer (Mapper.optimize_map's fused path: Mapper.py:314-333 each call).

        masks: {grid key: bool [X, Y, Z] (mapper.frustum_mask) or None = every voxel}.  On the first call
        (or a new key set) every listed grid gets a compact gradient sized for its CAPACITY (all of its
        voxels) plus a persistent row list, slot map and live row count; every call then rewrites those
        three in place from the masks (a cumsum compaction).  Adam segments carry the live count (ABI v19
        nslam_adam_seg.n_live, FusedAdam group "n_live"), so nothing an iteration launches depends on the
        selection's size: a hipGraph captured for one call replays for the next.  The compact gradients
        stay zero between iterations (the backward writes only live rows, Adam zeroes every row it reads).
        Returns {grid key: live row count (device int64 [1])}."""
        keys = tuple(sorted(masks))
        if getattr(self, "_cap_keys", None) != keys:
            self._cap = {}
            rows = {}
            for k in keys:
                n = self.c[k].numel() // 32
                full = torch.empty(n + 1, dtype=torch.int32, device=self.device)  # [n]: the dummy target
                full[:n] = torch.arange(n, dtype=torch.int32, device=self.device)
                self._cap[k] = (full, torch.full((1,), n, dtype=torch.int64, device=self.device),
                                torch.arange(n, dtype=torch.int32, device=self.device))
                rows[k] = full[:n]
            self.set_rows(rows, pad_rows=1)
            self._cap_keys = keys
            self.gall.zero_()
            self._clean = True
        for k in keys:
            full, n_live, ar = self._cap[k]
            n = ar.numel()
            m = masks[k]
            if m is None:
                full[:n].copy_(ar)
                self.slot[k].copy_(ar)
                n_live.fill_(n)
                continue
            m = m.permute(2, 1, 0).reshape(-1)  # [X, Y, Z] -> channels-last voxel order z*Y*X + y*X + x
            idx = torch.cumsum(m, 0, dtype=torch.int32) - 1
            self.slot[k].copy_(torch.where(m, idx, torch.full_like(idx, -1)))
            full.scatter_(0, torch.where(m, idx, torch.full_like(idx, n)).long(), ar)
            n_live.copy_(idx[-1:].to(torch.int64) + 1)
        return {k: self._cap[k][1] for k in keys}

    def live_rows(self, key):
        """(row list, live count) of a grid bound by bind_masks: the FusedAdam group's "rows" / "n_live"."""
        full, n_live, ar = self._cap[key]
        return full[:ar.numel()], n_live

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
                  on_branch=None, pts_parts=False, ordered_branches=False, on_pts=None):
        """Backward into the engine's gradient buffers, as independent launches ("branches") that write
        disjoint buffers:
          lean     every decoder's grid gradient (and d/dpts) from the forward's ReLU masks, ONE launch
                   (ABI v10 nslam_query_bwd_decoders; the trainable colour decoder included);
          wgrad    the colour decoder's parameter gradients (ABI v16 nslam_color_wgrad), which reads only
                   the forward's tapes and g_raw — so it runs beside the lean launch;
          others   a decoder with parameter gradients and no tape path (nslam_query_bwd_decoder each).
        With `concurrent` the branches run on separate streams (parallel branches of a captured hipGraph).

        pts_grad: also return d loss / d pts [N*S, 3] float64 (tracking, bundle adjustment): every
        decoder writes its share into its own buffer and the shares are summed afterwards (or returned
        as a list with pts_parts).
        on_branch(names, part): called on a branch's stream once what it updates is complete — "grids":
        the grids of the lean launch's decoders but the colour one; "all": the colour grid and the
        colour decoder, on the weight-gradient branch after it AND the lean launch (k_color_wgrad reads
        the colour grid: it is not rewritten before that kernel is done); "unit": a per-decoder launch's
        grid and parameters — the per-branch Adam of the mapping iteration.
        ordered_branches: the weight-gradient branch's on_branch starts only after the lean branch's
        on_branch work (not just the lean launch) — for collectives issued there on two communicators,
        which every rank must then run in the same order (distributed.ShardedAdamExchange).
        on_pts(parts): with pts_grad, called once every decoder's d/dpts share is written — on the lean
        launch's stream right after it when that launch forms all of them (bundle adjustment's camera
        gradient then runs beside the weight gradients, not after the join), else on the caller's stream
        after the join."""
        n = z.numel()
        self._clean = False
        concurrent = self.concurrent if concurrent is None else concurrent
        cfg = self._cfg(stage, ro, rd, z, grid_grads, dec_grads)
        cfg.need_pts_grad = int(bool(pts_grad))
        decs = list(ops._DEC_FOR_STAGE[stage])
        wgt = [d for d in decs if d in dec_grads]
        masks = self._saved is not None
        tape_color = "color" in wgt and masks and self._tape is not None
        lean = [d for d in decs if self.merge and masks and (d not in wgt or (d == "color" and tape_color))]
        others = [d for d in decs if d not in lean]
        gp = {d: torch.empty(n, 3, dtype=torch.float64, device=z.device) for d in decs} if pts_grad else None
        # units: (kind, decoder names) in enqueue order
        units = []
        if "color" in lean and "color" in wgt and n > 0:
            units.append(("wgrad", ["color"]))
        if lean:
            units.append(("lean", lean))
        units += [("one", [d]) for d in others]
        if not self.wgrad_first:
            units.sort(key=lambda u: u[0] == "wgrad")
        has_wgrad = any(u[0] == "wgrad" for u in units)
        merged_names = None
        # NSLAM_ADAM_MERGE=1: one Adam call after both branches, on the lean launch's stream
        merge_adam = (self.adam_merge and has_wgrad and on_branch is not None and not ordered_branches
                      and self.wgrad_first and concurrent and len(units) == 2 and units[1][0] == "lean")
        wgrad_st = None
        main = torch.cuda.current_stream(z.device)
        par = concurrent and len(units) > 1
        streams = [main]
        if par:
            while len(self._side) < len(units) - 1:
                self._side.append(torch.cuda.Stream(z.device))
            streams += self._side[:len(units) - 1]
        used = streams[1:]
        with ops._span("query_bwd"):
            for st in used:  # fork: every branch starts from the same point of the main stream
                st.wait_stream(main)
                for t in (ro, rd, z, g_raw, self._saved, self._tape):
                    if t is not None:
                        t.record_stream(st)
            for i, (kind, names) in enumerate(units):
                st = streams[i] if par else main
                with torch.cuda.stream(st):
                    if kind == "wgrad":
                        wsb = lib().nslam_query_bwd_decoder_workspace_size(ctypes.byref(cfg), _lib.DEC_COLOR, n)
                        ws = torch.empty(wsb, dtype=torch.uint8, device=z.device)
                        with ops._span("query_bwd.color_wgrad"):
                            rc = lib().nslam_color_wgrad(ctypes.byref(cfg), None, n, ptr(g_raw), ptr(ws), wsb,
                                                         st.cuda_stream)
                        check(rc, "nslam_color_wgrad")
                        wgrad_st = st  # (its update waits for the lean launch: see below)
                        if merge_adam:
                            if self._wg_ev is None:
                                self._wg_ev = torch.cuda.Event()
                            self._wg_ev.record(st)
                    elif kind == "lean":
                        lc = _lib.NslamQueryCfg.from_buffer_copy(cfg)  # grids (and d/dpts) only
                        gps = (ctypes.c_void_p * 4)()
                        mask = 0
                        for name in names:
                            d = ops._DEC_ID[name]
                            mask |= 1 << d
                            lc.dgrad[d] = _lib.NslamDecGrad()
                            if pts_grad:
                                gps[d] = ptr(gp[name])
                        with ops._span("query_bwd." + "+".join(names)):
                            rc = lib().nslam_query_bwd_decoders(ctypes.byref(lc), mask, None, n, ptr(g_raw), gps,
                                                                st.cuda_stream)
                        check(rc, "nslam_query_bwd_decoders")
                        if on_pts is not None and pts_grad and set(names) == set(decs):
                            for name in names:  # (allocated on the caller's stream)
                                gp[name].record_stream(st)
                            on_pts([gp[d] for d in decs])
                            on_pts = None
                        if has_wgrad and self._lean_ev is None:  # one persistent event (never destroyed mid-capture)
                            self._lean_ev = torch.cuda.Event()
                        if has_wgrad and not ordered_branches:
                            self._lean_ev.record(st)
                        if on_branch is not None and merge_adam and self.adam_on == "main":
                            merged_names = names  # (the merged Adam runs on the main stream after the join)
                        elif on_branch is not None and merge_adam:
                            # every update of the iteration in one Adam call on this stream, once the
                            # weight-gradient branch (its slab reduction; its colour-grid gathers) is done
                            st.wait_event(self._wg_ev)
                            on_branch(names, part="all")
                        elif on_branch is not None:
                            # the grids of this launch — but the colour grid, which k_color_wgrad reads (its
                            # colour feature) and which is updated on that branch once both are done.  A
                            # trainable decoder here without a weight-gradient branch (no points) still
                            # takes its Adam step (torch's Adam steps a parameter whose gradient is zero)
                            own = [d for d in names if not (d == "color" and has_wgrad)]
                            dec_here = not has_wgrad and any(d in wgt for d in own)
                            if own:
                                on_branch(own, part="all" if dec_here else "grids")
                        if has_wgrad and ordered_branches:
                            self._lean_ev.record(st)
                    else:
                        name = names[0]
                        d = ops._DEC_ID[name]
                        wsb = lib().nslam_query_bwd_decoder_workspace_size(ctypes.byref(cfg), d, n)
                        ws = torch.empty(wsb, dtype=torch.uint8, device=z.device) if wsb else None
                        with ops._span("query_bwd." + name):
                            rc = lib().nslam_query_bwd_decoder(ctypes.byref(cfg), d, 0, None, n, ptr(g_raw),
                                                               ptr(gp[name]) if pts_grad else None, ptr(ws), wsb,
                                                               st.cuda_stream)
                        check(rc, "nslam_query_bwd_decoder")
                        if on_branch is not None:
                            on_branch(names, part="unit")
                if pts_grad and st is not main:
                    for name in names:
                        gp[name].record_stream(st)
            if has_wgrad and on_branch is not None and not merge_adam:
                # the colour grid and the colour decoder, on the weight-gradient branch after its kernel
                # and after the lean launch (the colour grid's gradient; and no Adam may rewrite the grid
                # while k_color_wgrad still gathers from it)
                with torch.cuda.stream(wgrad_st):
                    wgrad_st.wait_event(self._lean_ev)
                    on_branch(["color"], part="all")
            for st in used:
                main.wait_stream(st)
            if on_pts is not None and pts_grad:
                on_pts([gp[d] for d in decs])
            if merged_names is not None:
                # NSLAM_ADAM_ON=main: the merged update on the main stream after the join (the weight
                # gradients ran on it; the join covers the lean launch), so the next iteration's forward
                # follows it on the same queue
                on_branch(merged_names, part="all")
        if not pts_grad:
            return None
        parts = [gp[d] for d in decs]
        if pts_parts:  # the per-decoder shares, for a consumer that sums them itself
            return parts
        out = parts[0]
        for g in parts[1:]:
            out += g
        return out

    # -- one iteration ---------------------------------------------------------------------------
    def draws(self, seed, world=1, rank=0):
        """The in-kernel pixel draws (ops.PixelDraws) of stream `seed`, made on first use."""
        key = (seed, world, rank)
        if self._draws is None or self._draws[0] != key:
            self._draws = (key, ops.PixelDraws(seed, self.device, world, rank, with_max=world > 1))
        return self._draws[1]

    def grads_for(self, stage, trainable_decoders):
        """(grid keys, decoder names) that receive gradients in `stage` (Mapper.py:335-341)."""
        decs = ops._DEC_FOR_STAGE[stage]
        keys = tuple(_GRID_OF[n] for n in decs)
        return keys, tuple(n for n in decs if n in trainable_decoders)

    def adam_grads(self, stage, trainable_decoders):
        """{parameter: its gradient buffer} of the stage (compact grids: [n_rows, 32], no padding)."""
        keys, dnames = self.grads_for(stage, trainable_decoders)
        g = {self.c[k]: self.ggrad[k] for k in keys}
        g.update({self.decs[n].param: self.decs[n].grad for n in dnames})
        return g

    def iteration(self, stage, frames, pix, n_per, hw, intrinsics, optimizer, trainable_decoders=("color",),
                  gt_max=None, allreduce=None, use_gt_in_sampler=True, exchange=None, n_kept=None, seed=0,
                  world=1, rank=0, prefetch=False, post_bwd=None):
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
        post_bwd(g_pts parts, rays_o, rays_d, z): the backward also forms d loss / d pts (every decoder's
        share, a list of [N*S, 3] float64) and this runs as soon as they are written (on the mask-only
        launch's stream, beside the weight gradients; query_bwd on_pts) — bundle adjustment's camera
        gradients and camera step (Mapper.py:346-363, 503-504).  Its work must be ordered before the
        next iteration by the join (it is: it runs on a stream the join covers).  Camera poses that a step changes in place make a prefetched batch
        stale (the version check cannot see a kernel's writes): the caller passes prefetch=False whenever
        its camera step can move them (Mapper: the colour stage, where their lr is not 0).
        """
        H, W = hw
        fx, fy, cx, cy = intrinsics
        keys, dnames = self.grads_for(stage, trainable_decoders)
        if exchange is not None and hasattr(exchange, "validate"):
            exchange.validate(self, keys, dnames)  # raises before anything of the iteration is enqueued
        draw = self.draws(seed, world, rank) if pix is None else None

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
            # A prefetched batch is only valid for the very frames (images and poses, unmodified) it was
            # gathered from: held by weak reference (identity — a new tensor that reuses a freed one's
            # address is not the same frame) and version counter.
            ftens = [t for f in frames for t in f]
            pkey = (stage, n_per, hw, use_gt_in_sampler, seed, world, rank)
            valid = (self._pre is not None and self._pre[0] == pkey and len(self._pre[1]) == len(ftens)
                     and all(r() is t and v == t._version for (r, v), t in zip(self._pre[1], ftens)))
            if not valid:
                first = rays()  # first call: this iteration's batch (set 0), then a same-shaped set 1
                self._pre = (pkey, [(weakref.ref(t), t._version) for t in ftens],
                             [first, [torch.empty_like(t) for t in first]])
                self._parity = 0
            cur, nxt = self._pre[2][self._parity], self._pre[2][1 - self._parity]
            self._parity ^= 1
            main = torch.cuda.current_stream(self.device)
            if self._pre_stream is None:
                if self.prefetch_stream == "lean" and self.wgrad_first and self.concurrent:
                    # the backward's first side stream (the mask-only launch's, with the weight-gradient
                    # branch enqueued first on the main stream): one side queue fewer in the iteration's
                    # graph; the prefetch is done long before that stream's backward work.  In any other
                    # topology that side stream carries the weight-gradient branch: the prefetch gets its own
                    if not self._side:
                        self._side.append(torch.cuda.Stream(self.device))
                    self._pre_stream = self._side[0]
                else:
                    self._pre_stream = torch.cuda.Stream(self.device)
            side = self._pre_stream

            def launch_prefetch():
                side.wait_stream(main)  # the previous iteration's backward has released `nxt`
                with torch.cuda.stream(side):
                    rays(out=nxt)  # the next iteration's batch, beside this iteration's render + backward

            if self.prefetch_at == "start":
                launch_prefetch()
            ro, rd, gd, gc, keep, z = cur
        else:
            ro, rd, gd, gc, keep, z = rays()
        mirror = hasattr(optimizer, "set_mirror")
        raw = self.query_fwd(stage, ro, rd, z, defer_occ=True, tape="color" in dnames)
        if side is not None and self.prefetch_at != "start":
            launch_prefetch()  # forks after the forward: beside the loss and the backward
        _, _, _, ray_loss, g_raw = ops.render_loss(raw, z, gd, gc, keep, mode="mapper", use_color=stage == "color",
                                                   w_color=self.w_color, occ_add=self.occ_add)
        if not self._clean:
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
        sharded = exchange is not None and hasattr(exchange, "branch")
        if sharded:
            # ZeRO-style exchange (distributed.ShardedAdamExchange): each backward branch's gradients are
            # reduce-scattered, this rank's shard stepped by Adam and the updated values all-gathered,
            # on that branch's stream as soon as it finishes — the exchange does the optimiser step
            def on_branch(names, part=None):
                exchange.branch(names, part, keys, dnames)
        elif exchange is None and allreduce is None and mirror:
            # one rank: each backward branch updates what it completes on its own stream — the lean
            # launch the middle / fine grid rows, the weight-gradient branch (once the lean launch is
            # done too) the colour grid and the colour decoder — so no Adam waits for the whole backward
            def on_branch(names, part=None):  # the decoders of one launch: one Adam call for their grids
                sub = {}                         # (part "grids" / "decoders": only those)
                for name in names:
                    if _GRID_OF[name] in keys and part != "decoders":
                        sub[self.c[_GRID_OF[name]]] = grads[self.c[_GRID_OF[name]]]
                    if name in dnames and part != "grids":
                        sub[self.decs[name].param] = grads[self.decs[name].param]
                if sub:
                    optimizer.step(grads=sub, zero_grad=clean)

        on_pts = (lambda parts: post_bwd(parts, ro, rd, z)) if post_bwd is not None else None
        self.query_bwd(stage, ro, rd, z, g_raw, keys, dnames, on_branch=on_branch, ordered_branches=sharded,
                       pts_grad=post_bwd is not None, pts_parts=True, on_pts=on_pts)
        if sharded:
            pass
        elif exchange is not None:  # frustum-compacted all-reduce (distributed.SparseGradExchange)
            exchange(keys, dnames)
        elif allreduce is not None:  # the grid gradients as one flat buffer, plus the decoder gradients
            allreduce([self.gbuf] + [self.decs[n].grad for n in dnames])
        if side is not None:  # join: the next call reads the prefetched set
            main.wait_stream(side)
        if on_branch is None:
            optimizer.step(grads=grads, zero_grad=clean)
        self._clean = clean and (not sharded or exchange.leaves_clean)
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
        pts → rays → c2w → cam                         nslam_cam_grad_step (closed form, include/nslam.h),
        Adam on the camera, loss sum, best pose          whose last workgroup also steps the camera (FusedAdam's
                                                       update, device step count) and keeps the best pose

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
        # ABI v23 nslam_cam_grad_step: with a FusedAdam over the camera alone, its step, the loss sum and the
        # best pose run in the camera-gradient launch's last workgroup (two launches fewer per iteration)
        self.cam_tail = True
        self._cam_ws = self._cam_ticket = None
        self._loss = None  # the last iteration's loss (device f64 scalar, overwritten by the next one)

    def n_window(self):
        h0, h1, w0, w1 = self.window
        return (h1 - h0) * (w1 - w0)

    @staticmethod
    def _tail_ok(optimizer, cam):
        """The fused camera tail applies to a FusedAdam stepping exactly this dense camera tensor."""
        if not isinstance(optimizer, ops.FusedAdam):
            return False
        ps = [p for g in optimizer.param_groups for p in g["params"]]
        return (len(ps) == 1 and ps[0] is cam and optimizer.param_groups[0].get("rows") is None
                and cam not in optimizer.mirrors and cam.is_contiguous() and cam.numel() == 7)

    def iteration(self, cam, depth, color, pix, optimizer, n=None, seed=0, best=None):
        """One camera iteration on frame (depth [H,W], color [H,W,3]) with pixel draws `pix`
        (int64 [n], select_uv indices into the edge-cropped window), or pix=None: n pixels drawn inside
        the gather kernel (uniform over the window, stream `seed`; capturable in a hipGraph).  cam: [7]
        leaf tensor whose .grad the optimizer reads.  Returns the loss (device f64 scalar) of the pose
        BEFORE the step: the kept rays' losses summed in a fixed order (nslam_loss_sum_best; a buffer the
        next call overwrites), which with best = (best_loss, best_cam) also keeps the best pose
        (Tracker.py:245-247) in the same launch."""
        fx, fy, cx, cy = self.intr
        n = pix.numel() if pix is not None else int(n)
        draw = self.eng.draws(seed) if pix is None else None
        if self._c2w is None:
            self._c2w = torch.empty(3, 4, dtype=torch.float32, device=cam.device)
        # get_camera_from_tensor inside the gather (ABI v21), which also leaves the pose in self._c2w for
        # the camera gradient
        c2w = self._c2w
        ro, rd, gd, gc, keep = ops.gather_rays([(depth, color, c2w, cam.detach())], pix, n, self.H, self.W,
                                               self.window, fx, fy, cx, cy, self.bound, draw=draw)
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
            if self._loss is None:
                self._loss = torch.empty((), dtype=torch.float64, device=cam.device)
            if self.cam_tail and self._tail_ok(optimizer, cam):
                ex, ex2, stp = optimizer.state_of(cam)
                adam = (ex, ex2, stp, optimizer.group_of(cam)["lr"], *optimizer.betas, optimizer.eps)
                bl, bc = (None, None) if best is None else (best[0], best[1])
                ops.cam_grad_step(cam.detach(), c2w, gps, z, rd, cam.grad, self._cam_ws, self._cam_ticket, adam,
                                  ray_loss, self._loss, bl, bc)
                return self._loss
            ops.cam_grad_parts(cam.detach(), c2w, gps, z, rd, cam.grad, self._cam_ws, self._cam_ticket)
        else:
            g_pts = self.eng.query_bwd("color", ro, rd, z, g_raw, (), (), pts_grad=True)
            # the whole pts → rays → c2w → 7-vector chain in one launch
            ops.cam_grad(cam.detach(), c2w, g_pts, z, rd, cam.grad)
        optimizer.step()
        # the loss of the pose before the step (its rays' losses) and, with `best`, the best-pose update in
        # one launch: the candidate is the 7-vector right after that step, as the reference keeps it
        # (optimize_cam_in_batch steps before Tracker.py:245-247 compares)
        if self._loss is None:
            self._loss = torch.empty((), dtype=torch.float64, device=cam.device)
        if best is None:
            ops.loss_sum_best(ray_loss, self._loss)
        else:
            ops.loss_sum_best(ray_loss, self._loss, best[0], cam.detach(), best[1])
        return self._loss


def frustum_rows(mask_xyz: torch.Tensor) -> torch.Tensor:
    """int32 voxel rows (z*Y*X + y*X + x, channels-last) of a get_mask_from_c2w mask [X, Y, Z]."""
    m = mask_xyz.permute(2, 1, 0).reshape(-1)
    return torch.nonzero(m).reshape(-1).to(torch.int32)
