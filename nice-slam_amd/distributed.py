"""Ray-sharded data parallelism for the mapping iteration (one process per GPU, RCCL over xGMI).

The reference is single-GPU.  Its per-iteration losses are sums over rays (Tracker.py:117-123,
Mapper.py:488-493), so gradients of ray shards add up exactly; the only cross-shard quantities
are the batch-global max(gt_depth) of the sampler (Renderer.py:109,144) — all-reduced here so a
shard samples exactly as the full batch would — and the tracker's median (handle_dynamic), which
would need an all-gather (tracking is not sharded).  Adam then runs replicated on identical
summed gradients, keeping every rank's map bit-identical.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def _collectives(group, force: bool) -> bool:
    """Whether an exchange issues its collectives: world > 1, or `force` with an initialised process
    group of any size (world 1 over RCCL: the collectives run as they would in a job, an identity
    on the data — the path the single-GPU box can exercise, bit-identical to no exchange)."""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return force or dist.get_world_size(group) > 1


def shard_range(n: int, rank: int, world: int):
    """Contiguous split of n rays over `world` ranks (first n % world ranks get one more)."""
    base, rem = divmod(n, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def global_max(x: torch.Tensor, group=None) -> torch.Tensor:
    """max over all ranks of max(x) (float scalar tensor on x's device; -inf for empty x)."""
    m = x.max().reshape(1).float() if x.numel() else torch.full((1,), float("-inf"), device=x.device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
    return m


def allreduce_grads(params, group=None, bucket_bytes: int = 64 << 20):
    """Sum .grad of `params` over ranks (see allreduce_tensors)."""
    allreduce_tensors([p.grad for p in params if p is not None and p.grad is not None], group, bucket_bytes)


def allreduce_tensors(grads, group=None, bucket_bytes: int = 64 << 20):
    """Sum tensors over ranks in place.  Large ones (feature-grid gradients; the fused engine
    passes all grids as one flat buffer) are reduced in place, small ones (decoder weights, camera
    7-vectors) are coalesced into buckets of ≤ bucket_bytes."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    small, size = [], 0

    def flush():
        nonlocal small, size
        if not small:
            return
        flat = torch.cat([g.reshape(-1) for g in small])
        dist.all_reduce(flat, group=group)
        off = 0
        for g in small:
            g.copy_(flat[off:off + g.numel()].view_as(g))
            off += g.numel()
        small, size = [], 0

    for g in grads:
        nb = g.numel() * g.element_size()
        if nb >= bucket_bytes // 4:
            dist.all_reduce(g, group=group)
        else:
            if size + nb > bucket_bytes:
                flush()
            small.append(g)
            size += nb
    flush()


class SparseGradExchange:
    """Frustum-compacted gradient all-reduce for the fused mapping engine (ray sharding).

    Adam only reads the frustum-selected rows of each grid gradient (Mapper.py:314-333,394-401,504;
    room0: ~5 % of the fine/colour grids), so the payload of the per-iteration exchange is those
    rows plus the dense decoder gradients: ~2.4 MiB instead of the 46 MiB dense room0 grids.
    nslam_rows_pack gathers them from the engine's flat grid-gradient buffer into one contiguous
    buffer, ONE all_reduce(SUM) sums it over ranks (RCCL over xGMI; capturable in a hipGraph), and
    nslam_rows_unpack writes it back.  Rows outside the frustum keep this rank's partial sums:
    Adam never reads them (the reference discards them at Mapper.py:511-519).

    rows: {grid key: int32 row indices} (the FusedAdam group "rows"); pack/unpack default to the
    HIP entry points (ops.rows_pack / ops.rows_unpack) and are injectable for CPU tests.
    force_collectives: issue the all-reduce at world size 1 too (RCCL on one GPU).
    """

    def __init__(self, engine, rows, group=None, pack=None, unpack=None, force_collectives=False):
        from . import ops
        self.engine, self.group = engine, group
        self.force = force_collectives
        self.pack = pack or ops.rows_pack
        self.unpack = unpack or ops.rows_unpack
        self.rows = self._flat_rows(rows)
        self._plan = {}
        self._gen = getattr(engine, "layout_gen", 0)

    def _flat_rows(self, rows):
        """{grid key: int32 rows offset into the engine's flat (dense) grid-gradient buffer}."""
        offs, off = {}, 0
        for k, v in self.engine.c.items():  # flat buffer order = engine.ggrad order
            offs[k] = off
            off += v.numel() // 32
        return {k: (r.to(torch.int64) + offs[k]).to(torch.int32) for k, r in rows.items()}

    def validate(self, engine, keys, dnames):
        """engine.MappingEngine.iteration calls this before it enqueues anything: the cached plans hold
        views of the engine's gradient buffers, which set_rows reallocates.  After set_rows, a grid this
        exchange sums by row list must be compact in the engine's new rows (whose compact buffer then
        carries exactly the rows Adam reads); a grid that went back to a dense gradient would be summed
        on the old rows while Adam reads others — the ranks would diverge silently, so that raises."""
        if engine is not self.engine:
            raise ValueError("SparseGradExchange: built for another engine")
        gen = getattr(engine, "layout_gen", 0)
        if gen != self._gen:
            cur = getattr(engine, "rows", {})
            stale = sorted(k for k in self.rows if k not in cur)
            if stale:
                raise RuntimeError(f"SparseGradExchange: the engine's gradient rows changed (set_rows) and {stale} "
                                   "no longer have compact gradients; build a new exchange for the new rows")
            self.rows = self._flat_rows(cur)
            self._plan.clear()  # (views of the old buffers)
            self._gen = gen

    def plan(self, keys, dnames):
        """(flat row list, [(decoder grad, offset)], payload buffer) for the grids in `keys` and
        the decoders `dnames` (cached per stage).  An engine with frustum-compacted gradients
        (engine.rows) already holds exactly the rows to exchange: its compact grid gradients
        join the decoder gradients as plain copies (row list empty)."""
        k = (tuple(keys), tuple(dnames))
        if k not in self._plan:
            dev = self.engine.gbuf.device
            compact = [g for g in keys if g in getattr(self.engine, "rows", {})]
            rl = [self.rows[g] for g in keys if g in self.rows and g not in compact]
            rows = torch.cat(rl) if rl else torch.zeros(0, dtype=torch.int32, device=dev)
            tails, off = [], rows.numel() * 32
            for g in compact:
                t = self.engine.ggrad[g]
                tails.append((t, off))
                off += t.numel()
            for n in dnames:
                g = self.engine.decs[n].grad
                tails.append((g, off))
                off += g.numel()
            span = None
            if not rows.numel() and tails:  # compact pieces back to back in one buffer: exchange in place
                pieces = sorted(((t.data_ptr(), t.numel(), t) for t, _ in tails), key=lambda q: q[0])
                if all(a[0] + a[1] * 4 == b[0] for a, b in zip(pieces, pieces[1:])):
                    base = pieces[0][2]
                    span = base.as_strided((sum(p[1] for p in pieces),), (1,))
            buf = span if span is not None else torch.empty(off, dtype=torch.float32, device=dev)
            self._plan[k] = (rows, tails if span is None else [], buf)
        return self._plan[k]

    def payload_bytes(self, keys, dnames):
        return self.plan(keys, dnames)[2].numel() * 4

    def __call__(self, keys, dnames):
        rows, tails, buf = self.plan(keys, dnames)  # no rows, no tails: buf is the gradients themselves
        gbuf = self.engine.gbuf
        if rows.numel():
            self.pack(gbuf, rows, None, buf)
        for g, off in tails:
            self.pack(None, None, g.reshape(-1), buf[off:off + g.numel()])
        if _collectives(self.group, self.force):
            from .ops import _span
            with _span("collective.all_reduce"):
                dist.all_reduce(buf, group=self.group)
        if rows.numel():
            self.unpack(buf, rows, gbuf, None)
        for g, off in tails:
            self.unpack(buf[off:off + g.numel()], None, None, g.reshape(-1))


def _storage(t):
    """A dense tensor's elements in storage order, as a view (a channels-last grid's [Z][Y][X][C])."""
    if t.dim() == 5 and not t.is_contiguous():
        return t.permute(0, 2, 3, 4, 1).reshape(-1)
    return t.reshape(-1)


class ShardedAdamExchange:
    """The ray-sharded mapping iteration's gradient exchange with the optimiser step sharded across
    ranks (ZeRO-1 style; SURVEY §8(e), Mapper.py:503-504 on the summed gradients):

        reduce-scatter  the branch's compact gradient span (frustum rows of its grids, or a decoder's
                        gradient): rank r receives the summed shard r            (in place)
        Adam            on shard r only: this rank's slices of the row-masked grid segments / of the
                        decoder (nslam_adam_step over explicit sub-segments; its Adam state is only
                        ever touched there, the rest stays zero)
        all-gather      the updated values of every shard (rows gathered from the grids, decoder
                        parameters), then written back (nslam_rows_unpack)    (in place)

    The bytes on the wire are an all-reduce's (a reduce-scatter plus an all-gather of the same span)
    and each rank runs 1/N of the Adam work, which the replicated design ran N times.  It runs per
    backward BRANCH (engine.MappingEngine.iteration calls branch() on the branch's stream right after
    it): the grids' exchange starts when the lean backward launch completes, while the colour decoder's
    weight gradients are still running; the decoder's exchange follows them on their own stream, over a
    second process group (two communicators: collectives from two streams never share one).

    The engine's compact gradients are padded to whole shards (engine.set_rows(pad_rows=world)); the
    exchange zeroes every gradient entry it consumed, so the next iteration needs no memset.  The two
    branches' collectives run on two communicators from two streams, so the engine orders them
    (query_bwd(ordered_branches=True): the weight-gradient branch's exchange starts after the lean
    branch's) and every rank issues them in the same order.  Supported: the colour decoder as the only
    trainable decoder, with the engine's merged mask-only launch (its parameters then come from the
    weight-gradient branch); validate() raises before an iteration enqueues anything otherwise.
    force_collectives: issue the collectives at world size 1 too (RCCL on one GPU: identities).
    pack / unpack / adam_slices default to the HIP entry points and are injectable for CPU tests."""

    leaves_clean = True

    def __init__(self, engine, optimizer, group=None, group_dec=None, pack=None, unpack=None, adam_slices=None,
                 force_collectives=False):
        from . import ops
        self.engine, self.opt, self.group = engine, optimizer, group
        init = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if init else 1
        self.rank = dist.get_rank(group) if init else 0
        self.coll = _collectives(group, force_collectives)
        if not engine.merge:
            raise ValueError("ShardedAdamExchange needs the engine's merged mask-only backward (engine.merge)")
        if group_dec is None and self.coll:
            group_dec = dist.new_group(dist.get_process_group_ranks(group) if group is not None else None)
        self.group_dec = group_dec
        self.pack = pack or ops.rows_pack
        self.unpack = unpack or ops.rows_unpack
        self.adam_slices = adam_slices or self._adam_hip
        if engine.pad_rows != self.world:
            engine.set_rows(engine.rows, pad_rows=self.world)
        self._plans = {}
        self._gen = engine.layout_gen

    def validate(self, engine, keys, dnames):
        """Raise, before an iteration enqueues any kernel or collective, on what branch() cannot run."""
        if engine is not self.engine:
            raise ValueError("ShardedAdamExchange: built for another engine")
        if engine.layout_gen != self._gen or engine.pad_rows != self.world:
            raise RuntimeError("ShardedAdamExchange: the engine's gradient rows changed (MappingEngine.set_rows) "
                               "after the exchange was built; its shards and the optimiser's Adam state belong "
                               "to the old rows — build a new optimiser and exchange")
        if not engine.merge:
            raise ValueError("ShardedAdamExchange needs the engine's merged mask-only backward (engine.merge)")
        if any(n != "color" for n in dnames):
            raise ValueError(f"ShardedAdamExchange: trainable decoders {list(dnames)}: only the colour decoder "
                             "(its weight gradients in nslam_color_wgrad) is supported; use SparseGradExchange")

    # -- layout ---------------------------------------------------------------------------------
    def _span(self, pieces):
        """The contiguous view over `pieces` (tensors adjacent in the engine's flat buffer, in order)."""
        for a, b in zip(pieces, pieces[1:]):
            if a.data_ptr() + a.numel() * 4 != b.data_ptr():
                raise ValueError("ShardedAdamExchange: the branch's gradients are not one contiguous span")
        return pieces[0].as_strided((sum(p.numel() for p in pieces),), (1,))

    def _plan(self, gkeys, dnames):
        """(gradient span, value buffer, [(param, rows or None, n valid, offset in span, decoder)], chunk)
        over the grids `gkeys` then the decoders `dnames` (adjacent in the engine's flat buffer)."""
        key = (gkeys, dnames)
        if key not in self._plans:
            eng = self.engine
            pieces = [eng.ggrad_pad[k] for k in gkeys] + [eng.dgrad_pad[n] for n in dnames]
            segs = [(eng.c[k], eng.rows.get(k), eng.ggrad[k].numel(), None) for k in gkeys]
            segs += [(eng.decs[n].param, None, eng.decs[n].param.numel(), n) for n in dnames]
            span = self._span(pieces)
            if span.numel() % (self.world * 32):
                raise ValueError("ShardedAdamExchange: span not padded to whole shards")
            chunk = span.numel() // self.world
            vals = torch.empty_like(span)
            off, placed = 0, []
            for (p, rows, n, dec), piece in zip(segs, pieces):
                placed.append((p, rows, n, off, dec))
                off += piece.numel()
            self._plans[key] = (span, vals, placed, chunk)
        return self._plans[key]

    # -- collectives (gloo has no in-place reduce-scatter of device tensors: all-reduce, same shard) --
    def _reduce_scatter(self, span, chunk, group):
        own = span[self.rank * chunk:(self.rank + 1) * chunk]
        if not self.coll:
            return own
        from .ops import _span
        with _span("collective.reduce_scatter"):
            if dist.get_backend(group) == "gloo":
                dist.all_reduce(span, group=group)
            else:
                dist.reduce_scatter_tensor(own, span, group=group)
        return own

    def _all_gather(self, vals, chunk, group):
        if not self.coll:
            return
        own = vals[self.rank * chunk:(self.rank + 1) * chunk]
        from .ops import _span
        with _span("collective.all_gather"):
            if dist.get_backend(group) == "gloo":
                parts = list(vals.split(chunk))
                dist.all_gather(parts, own.clone(), group=group)
            else:
                dist.all_gather_into_tensor(vals, own, group=group)

    # -- one branch -----------------------------------------------------------------------------
    def branch(self, names, part, keys, dnames):
        """One backward branch's exchange + sharded Adam (engine.MappingEngine.query_bwd's on_branch):
        part "grids" (the lean launch: its grids, over `group`) or "all" (the weight-gradient branch:
        the colour grid and decoder, one span, over `group_dec`)."""
        if part not in ("grids", "all"):  # (validate() rules this out before the iteration starts)
            raise ValueError(f"ShardedAdamExchange: unsupported backward branch {part!r}")
        gk = tuple(k for k in ("grid_" + n for n in names) if k in keys)
        dk = tuple(n for n in names if n in dnames) if part == "all" else ()
        if not gk and not dk:
            return
        group = self.group if part == "grids" else self.group_dec
        span, vals, placed, chunk = self._plan(gk, dk)
        own0, own1 = self.rank * chunk, (self.rank + 1) * chunk
        self._reduce_scatter(span, chunk, group)
        # Adam on this rank's shard: the sub-segment of every piece that overlaps [own0, own1)
        slices = []
        for p, rows, n, off, dec in placed:
            a, b = max(own0, off), min(own1, off + n)  # (the piece's padding is never stepped)
            if a < b:
                slices.append((p, rows, a - off, b - off, a))
        self.adam_slices(slices, span, ("sharded",) + gk + dk)
        span.zero_()  # every entry consumed (the next iteration accumulates into zeros)
        # the shard's updated values, all-gathered, written back on every rank
        for p, rows, a0, b0, a in slices:
            if rows is not None:
                self.pack(_storage(p.data), rows[a0 // 32:b0 // 32], None, vals[a:a + (b0 - a0)])
            else:
                vals[a:a + (b0 - a0)].copy_(_storage(p.data)[a0:b0])
        self._all_gather(vals, chunk, group)
        for p, rows, n, off, dec in placed:
            if rows is not None:
                self.unpack(vals[off:off + n], rows, _storage(p.data), None)
            else:
                _storage(p.data).copy_(vals[off:off + n])
                if dec is not None:
                    self.engine.decs[dec].repack()  # the MFMA-packed copy of the updated decoder

    def _adam_hip(self, slices, span, key):
        """nslam_adam_step over this rank's slices: a row-masked grid segment takes whole rows a0/32 ..
        b0/32 of its row list (compact gradient in the span, its compact Adam state from a0); a dense
        one (a decoder, or a dense channels-last grid) elements a0 .. b0 of its storage."""
        from . import _lib
        from ._lib import ptr
        segs = []
        for p, rows, a0, b0, a in slices:
            ex, ex2, step = self.opt.state_of(p)
            s = _lib.NslamAdamSeg()
            s.grad = ptr(span) + a * 4
            s.exp_avg, s.exp_avg_sq, s.step = ptr(ex) + a0 * 4, ptr(ex2) + a0 * 4, ptr(step)
            s.lr = float(self.opt.group_of(p)["lr"])
            if rows is not None:
                s.param, s.rows, s.n, s.row_len, s.grad_rows = ptr(p.data), ptr(rows) + (a0 // 32) * 4, (b0 - a0) // 32, 32, 1
            else:
                s.param, s.rows, s.n, s.row_len = ptr(p.data) + a0 * 4, None, b0 - a0, 0
            segs.append(s)
        self.opt.step_segments(segs, key)

    def payload_bytes(self, keys, dnames):
        """Bytes each rank sends + receives per iteration ~ 2 (N-1)/N of these (reduce-scatter and
        all-gather of the padded spans)."""
        eng = self.engine
        g = sum(eng.ggrad_pad[k].numel() for k in keys if k in eng.ggrad_pad)
        d = sum(eng.dgrad_pad[n].numel() for n in dnames)
        return (g + d) * 4


def optimizer_params(opt):
    return [p for grp in opt.param_groups for p in grp["params"]]
