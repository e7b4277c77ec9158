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
    """

    def __init__(self, engine, rows, group=None, pack=None, unpack=None):
        from . import ops
        self.engine, self.group = engine, group
        self.pack = pack or ops.rows_pack
        self.unpack = unpack or ops.rows_unpack
        offs, off = {}, 0
        for k, v in engine.c.items():  # flat buffer order = engine.ggrad order
            offs[k] = off
            off += v.numel() // 32
        self.rows = {k: (r.to(torch.int64) + offs[k]).to(torch.int32) for k, r in rows.items()}
        self._plan = {}

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
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(self.group) > 1:
            dist.all_reduce(buf, group=self.group)
        if rows.numel():
            self.unpack(buf, rows, gbuf, None)
        for g, off in tails:
            self.unpack(buf[off:off + g.numel()], None, None, g.reshape(-1))


def optimizer_params(opt):
    return [p for grp in opt.param_groups for p in grp["params"]]
