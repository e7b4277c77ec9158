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
usage: python tools/probes/touched_rows.py [--world 8] [--configs apartment,stress]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--configs", default="apartment,stress")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    cfgs = {"apartment": (bench.APARTMENT, False), "stress": (bench.STRESS, True), "room0": (bench.ROOM0, False)}
    for name in args.configs.split(","):
        cfg, di = cfgs[name]
        print(json.dumps(measure(name, cfg, dev, args.world, di)), flush=True)


if __name__ == "__main__":
    main()
