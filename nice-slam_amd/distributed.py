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


def optimizer_params(opt):
    return [p for grp in opt.param_groups for p in grp["params"]]
