"""Grid-gradient scatter statistics of the room0 colour-stage mapping batch: per grid, how many
corner contributions a 32-point tile issues (8 per point), how many remain after merging runs of
identical cells (what the kernels do), after merging identical corner rows per tile, and how
many fall on frustum-selected rows (the only rows Adam reads, Mapper.py:314-333).

python tools/probes/scatter_stats.py   (on the GPU box)
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def corners(pts, lo, hi, dims):
    """channels-last row of the 8 trilinear corners of each point (align_corners=True, border)."""
    Z, Y, X = dims
    n = (pts - lo) / (hi - lo) * 2 - 1
    sz = torch.tensor([X - 1, Y - 1, Z - 1], dtype=pts.dtype, device=pts.device)
    f = ((n + 1) / 2 * sz).clamp(min=0)
    f = torch.minimum(f, sz)
    i0 = f.floor().long()
    i0 = torch.minimum(i0, (sz - 1).long().clamp(min=0))
    rows = []
    for dz in (0, 1):
        for dy in (0, 1):
            for dx in (0, 1):
                x, y, z = i0[:, 0] + dx, i0[:, 1] + dy, i0[:, 2] + dz
                rows.append((z * Y + y) * X + x)
    return torch.stack(rows, 1), (i0[:, 2] * Y + i0[:, 1]) * X + i0[:, 0]


def main():
    dev = torch.device("cuda:0")
    P = bench.pkg()
    sc = bench.Room0Scene(dev, 0, path="fused")
    cfg = sc.cfg
    F, H, W = cfg["window"], cfg["H"], cfg["W"]
    n = cfg["pixels"] // F
    pix = torch.randint(H * W, (F * n,), device=dev)
    ro, rd, gd, gc, keep = P.ops.gather_rays(sc.frames, pix, n, H, W, (0, H, 0, W), cfg["fx"], cfg["fy"], cfg["cx"],
                                             cfg["cy"], sc.bound)
    z = P.ops.sample_z(ro, rd, gd, sc.bound, 32, 16)
    # the same rays in pixel-Morton order within each frame (a permutation of the iid draws)
    u, v = (pix % W).long(), (pix // W).long()
    mort = torch.zeros_like(u)
    for bit in range(11):
        mort |= ((u >> bit) & 1) << (2 * bit) | ((v >> bit) & 1) << (2 * bit + 1)
    frame = torch.arange(F * n, device=dev) // n
    order = torch.argsort(frame * (1 << 24) + mort)
    for label, perm in (("draw order", None), ("morton order", order)):
        print(f"== rays in {label}", flush=True)
        stats(sc, ro, rd, z, keep, perm, dev)


def stats(sc, ro, rd, z, keep, perm, dev):
    if perm is not None:
        ro, rd, z, keep = ro[perm], rd[perm], z[perm], keep[perm]
    pts = (ro.double()[:, None] + rd.double()[:, None] * z[..., None]).reshape(-1, 3)
    kept = keep.bool().repeat_interleave(48)
    lo, hi = sc.bound[:, 0].to(dev), sc.bound[:, 1].to(dev)
    for key in ("grid_middle", "grid_fine", "grid_color"):
        dims = sc.grids[key].shape[2:]
        rows, cell = corners(pts, lo, hi, dims)
        m = torch.zeros(dims[0] * dims[1] * dims[2], dtype=torch.bool, device=dev)
        m[sc.rows[key].long()] = True
        T = rows.shape[0] // 32
        rt, ct, kt = rows[:T * 32].view(T, 32, 8), cell[:T * 32].view(T, 32), kept[:T * 32].view(T, 32)
        total = int(kt.sum()) * 8
        new_run = torch.ones_like(ct, dtype=torch.bool)
        new_run[:, 1:] = ct[:, 1:] != ct[:, :-1]
        runs = int((new_run & kt).sum()) * 8
        uniq = {}
        for g in (1, 4, 8, 32):
            u = 0
            for t in range(0, T, g):
                r = rt[t:t + g][kt[t:t + g]].reshape(-1)
                u += int(torch.unique(r).numel())
            uniq[g] = u
        inmask = int((m[rt.reshape(-1)].view(T, 32, 8) & kt[..., None]).sum())
        # flush wave-instructions of the uniform walk (one per corner pair (2j, 2j+1) with a nonzero
        # frustum weight), run-merge only vs with the carry-over of shared corners
        ins_run, ins_carry = walk_counts(rt, ct, kt, m, dims)
        us = "  ".join(f"{g}-tile {u} ({u / total:.2f})" for g, u in uniq.items())
        print(f"{key:12s} dims {tuple(dims)} frustum rows {int(m.sum())}/{m.numel()}  corner contributions {total}  "
              f"after run-merge {runs} ({runs / total:.2f})  unique rows per {us}  "
              f"on frustum rows {inmask} ({inmask / total:.2f})  flush instructions run-merge {ins_run} "
              f"carry {ins_carry} ({ins_carry / max(ins_run, 1):.2f})", flush=True)


def walk_counts(rt, ct, kt, m, dims):
    Z, Y, X = dims
    rt, ct, kt, m = rt.cpu().numpy(), ct.cpu().numpy(), kt.cpu().numpy(), m.cpu().numpy()
    n_run = n_carry = 0
    for t in range(rt.shape[0]):
        live_run = [False] * 8
        live_c = [False] * 8
        cur = None
        for p in range(32):
            c = int(ct[t, p])
            on = [bool(kt[t, p] and m[rt[t, p, k]]) for k in range(8)]
            if c != cur:
                if cur is not None:
                    n_run += sum(1 for j in range(4) if live_run[2 * j] or live_run[2 * j + 1])
                    cz, cy, cx = cur // (Y * X), (cur // X) % Y, cur % X
                    nz, ny, nx = c // (Y * X), (c // X) % Y, c % X
                    ax, ay, az = nx - cx, ny - cy, nz - cz
                    adj = max(abs(ax), abs(ay), abs(az)) <= 1
                    flushed = [False] * 8
                    new = [False] * 8
                    for k in range(8):
                        dx, dy, dz = k & 1, (k >> 1) & 1, k >> 2
                        mx, my, mz = dx - ax, dy - ay, dz - az
                        if adj and 0 <= mx <= 1 and 0 <= my <= 1 and 0 <= mz <= 1:
                            new[mx + 2 * my + 4 * mz] = live_c[k]
                        else:
                            flushed[k] = live_c[k]
                    n_carry += sum(1 for j in range(4) if flushed[2 * j] or flushed[2 * j + 1])
                    live_c = new
                else:
                    live_c = [False] * 8
                live_run = [False] * 8
                cur = c
            live_run = [a or b for a, b in zip(live_run, on)]
            live_c = [a or b for a, b in zip(live_c, on)]
        n_run += sum(1 for j in range(4) if live_run[2 * j] or live_run[2 * j + 1])
        n_carry += sum(1 for j in range(4) if live_c[2 * j] or live_c[2 * j + 1])
    return n_run, n_carry


if __name__ == "__main__":
    main()
