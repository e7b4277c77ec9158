"""Fraction of the frustum rows a ray-sharded mapping iteration actually touches (SURVEY §8(e),
VERDICT r4 item 4): does a touched-row exchange (OR-reduced row bitmap + compacted rows) beat
exchanging every frustum row?

For configs[3] (Apartment, 5000 px per rank) and configs[4] (stress, 512^3 grids, 65536 px per
rank), 8 ranks: each rank's slice of the global pixel batch is drawn exactly as the product draws it
(ops.PixelDraws(world=8, rank=r): same seed, rank r's slots), gathered and sampled on the device
(ops.gather_rays, ops.sample_z with the global max(gt_depth)); every sample of a kept ray marks the 8
trilinear corners of its cell in each grid (decoder.py:168-175, align_corners=True, border clamp).
Printed per grid: frustum rows (Mapper.py:314-333), rows touched by one rank (mean over ranks) and by
the union over the 8 ranks, as fractions of the frustum rows, and the resulting exchange bytes.

--split coherent: the rank-coherent ray split.  Every rank draws the SAME global
batch (world x pixels-per-rank per frame, one torch.randint stream) and keeps the rays whose pixel lies
in its image tile (a tx x ty tiling of the H x W image, tx * ty = world); the union over ranks is the
global batch, so the iteration's maths is the random split's.  Over --iters iterations of the same
window (a mapping call), it reports per grid: rows one rank touches per iteration; rows touched by
more than one rank in the same iteration (what a reduction must sum); and, over the call, each rank's
REGION (rows it touched in any iteration) and the rows in two or more regions (the rows an
owner-partitioned exchange must keep consistent between ranks every iteration).
usage: python tools/probes/touched_rows.py [--world 8] [--configs apartment,stress] [--split coherent --iters 6]
"""
import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def corner_rows(pts, lo, hi, dims):
    """int64 rows (z*Y + y)*X + x of the 8 corners of every point's cell (out-of-range corners dropped)."""
    Z, Y, X = dims
    n = (X, Y, Z)
    idx, ok = [], []
    for a in range(3):
        c = (((pts[:, a] - lo[a]) / (hi[a] - lo[a])) * 2.0 - 1.0).float()
        u = ((c + 1.0) / 2.0 * (n[a] - 1)).clamp(0, n[a] - 1)
        i0 = torch.floor(u).long()
        idx.append((i0, i0 + 1))
        ok.append((torch.ones_like(i0, dtype=torch.bool), i0 + 1 <= n[a] - 1))
    rows = []
    for k in range(8):
        dx, dy, dz = k & 1, (k >> 1) & 1, k >> 2
        m = ok[0][dx] & ok[1][dy] & ok[2][dz]
        r = (idx[2][dz] * Y + idx[1][dy]) * X + idx[0][dx]
        rows.append(r[m])
    return torch.cat(rows)


def measure(name, cfg, dev, world, device_init):
    P = bench.pkg()
    scene = bench.Room0Scene(dev, 0, cfg=dict(cfg), path="fused", device_init=device_init)
    F, H, W = cfg["window"], cfg["H"], cfg["W"]
    n = cfg["pixels"] // F
    bound = scene.bound.to(torch.float64)
    lo, hi = [float(v) for v in bound[:, 0]], [float(v) for v in bound[:, 1]]
    keys = [k for k in ("grid_middle", "grid_fine", "grid_color") if k in scene.rows]
    frustum, union, per_rank = {}, {}, {k: [] for k in keys}
    for k in keys:
        nvox = scene.grids[k][0, 0].numel()
        m = torch.zeros(nvox, dtype=torch.bool, device=dev)
        m[scene.rows[k].long()] = True
        frustum[k] = m
        union[k] = torch.zeros(nvox, dtype=torch.bool, device=dev)
    for r in range(world):
        draw = P.ops.PixelDraws(1000, dev, world, r, with_max=True)
        ro, rd, gd, gc, keep = P.ops.gather_rays(scene.frames, None, n, H, W, (0, H, 0, W), cfg["fx"], cfg["fy"],
                                                 cfg["cx"], cfg["cy"], scene.bound, draw=draw)
        z = P.ops.sample_z(ro, rd, gd, scene.bound, cfg["n_strat"], cfg["n_surf"], False, gt_max=draw.gt_max)
        kb = keep.bool()
        pts = (ro[kb, None, :].double() + rd[kb, None, :].double() * z[kb][..., None]).reshape(-1, 3)
        for k in keys:
            rows = corner_rows(pts, lo, hi, tuple(scene.grids[k].shape[2:]))
            t = torch.zeros_like(union[k])
            t[rows] = True
            t &= frustum[k]
            per_rank[k].append(int(t.sum()))
            union[k] |= t
        del pts
    out = {"config": name, "world": world, "pixels_per_rank": cfg["pixels"], "grids": {}}
    tot_f = tot_u = 0
    for k in keys:
        nf = int(frustum[k].sum())
        nu = int(union[k].sum())
        tot_f += nf
        tot_u += nu
        out["grids"][k] = {"frustum_rows": nf, "rank_touched_mean": sum(per_rank[k]) / world,
                           "rank_touched_frac": sum(per_rank[k]) / world / max(nf, 1),
                           "union_touched": nu, "union_frac": nu / max(nf, 1)}
    out["frustum_bytes"] = tot_f * 128
    out["union_bytes"] = tot_u * 128
    out["union_frac_all"] = tot_u / max(tot_f, 1)
    del scene
    torch.cuda.empty_cache()
    return out


def tiling(world):
    """(tx, ty): the most square tx x ty = world tiling, tx >= ty (the image is wider than tall)."""
    ty = max(d for d in range(1, int(world ** 0.5) + 1) if world % d == 0)
    return world // ty, ty


def measure_coherent(name, cfg, dev, world, device_init, iters):
    P = bench.pkg()
    scene = bench.Room0Scene(dev, 0, cfg=dict(cfg), path="fused", device_init=device_init)
    F, H, W = cfg["window"], cfg["H"], cfg["W"]
    n = cfg["pixels"] // F  # pixels per rank per frame; the global batch has n * world per frame
    tx, ty = tiling(world)
    bound = scene.bound.to(torch.float64)
    lo, hi = [float(v) for v in bound[:, 0]], [float(v) for v in bound[:, 1]]
    keys = [k for k in ("grid_middle", "grid_fine", "grid_color") if k in scene.rows]
    nvox = {k: scene.grids[k][0, 0].numel() for k in keys}
    frustum = {}
    for k in keys:
        m = torch.zeros(nvox[k], dtype=torch.bool, device=dev)
        m[scene.rows[k].long()] = True
        frustum[k] = m
    region = {k: torch.zeros(world, nvox[k], dtype=torch.bool, device=dev) for k in keys}
    per_rank, multi, rays = {k: [] for k in keys}, {k: [] for k in keys}, []
    g = torch.Generator(device=dev).manual_seed(1000)
    for it in range(iters):
        pix = torch.randint(H * W, (F, n * world), device=dev, generator=g)
        tile = ((pix // W) * ty // H) * tx + (pix % W) * tx // W  # rank owning each pixel
        # the global batch's max(gt_depth) over kept rays (what every rank's sampler uses)
        ro, rd, gd, gc, keep = P.ops.gather_rays(scene.frames, pix.reshape(-1), n * world, H, W, (0, H, 0, W),
                                                 cfg["fx"], cfg["fy"], cfg["cx"], cfg["cy"], scene.bound)
        gmax = gd[keep.bool()].max().reshape(1)
        cnt = {k: torch.zeros(nvox[k], dtype=torch.int32, device=dev) for k in keys}
        nr = []
        for r in range(world):
            sel = (tile.reshape(-1) == r)
            kb = keep.bool() & sel
            nr.append(int(kb.sum()))
            z = P.ops.sample_z(ro[kb].contiguous(), rd[kb].contiguous(), gd[kb].contiguous(), scene.bound,
                               cfg["n_strat"], cfg["n_surf"], False, gt_max=gmax)
            pts = (ro[kb, None, :].double() + rd[kb, None, :].double() * z[..., None]).reshape(-1, 3)
            for k in keys:
                t = torch.zeros(nvox[k], dtype=torch.bool, device=dev)
                t[corner_rows(pts, lo, hi, tuple(scene.grids[k].shape[2:]))] = True
                t &= frustum[k]
                per_rank[k].append(int(t.sum()))
                cnt[k] += t.int()
                region[k][r] |= t
            del pts
        rays.append(nr)
        for k in keys:
            multi[k].append(int((cnt[k] > 1).sum()))
    out = {"config": name, "split": "coherent", "world": world, "tiling": [tx, ty], "iters": iters,
           "pixels_per_rank": cfg["pixels"], "kept_rays_per_rank_min_max": [min(min(r) for r in rays),
                                                                            max(max(r) for r in rays)], "grids": {}}
    tot = {"frustum": 0, "rank": 0.0, "multi": 0.0, "region_shared": 0, "union": 0}
    for k in keys:
        nf = int(frustum[k].sum())
        reg = region[k].int().sum(0)
        shared = int((reg > 1).sum())
        un = int((reg > 0).sum())
        rk = sum(per_rank[k]) / len(per_rank[k])
        mu = sum(multi[k]) / len(multi[k])
        out["grids"][k] = {"frustum_rows": nf, "rank_touched_per_iter": rk, "rank_touched_frac": rk / max(nf, 1),
                           "multi_touched_per_iter": mu, "multi_frac": mu / max(nf, 1),
                           "union_over_call": un, "region_shared_rows": shared, "region_shared_frac": shared / max(nf, 1),
                           "region_rows_per_rank": int(region[k].sum()) / world}
        tot["frustum"] += nf
        tot["rank"] += rk
        tot["multi"] += mu
        tot["region_shared"] += shared
        tot["union"] += un
    out["bytes"] = {"frustum_rows": tot["frustum"] * 128, "rank_touched_per_iter": tot["rank"] * 128,
                    "multi_touched_per_iter": tot["multi"] * 128, "region_shared_rows": tot["region_shared"] * 128,
                    "union_over_call": tot["union"] * 128}
    del scene
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--configs", default="apartment,stress")
    ap.add_argument("--split", choices=("random", "coherent"), default="random")
    ap.add_argument("--iters", type=int, default=6)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    cfgs = {"apartment": (bench.APARTMENT, False), "stress": (bench.STRESS, True), "room0": (bench.ROOM0, False)}
    for name in args.configs.split(","):
        cfg, di = cfgs[name]
        if args.split == "coherent":
            print(json.dumps(measure_coherent(name, cfg, dev, args.world, di, args.iters)), flush=True)
        else:
            print(json.dumps(measure(name, cfg, dev, args.world, di)), flush=True)


if __name__ == "__main__":
    main()
