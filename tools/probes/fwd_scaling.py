"""Forward query time vs batch size / stage / launch form (latency- vs throughput-bound probe).

python tools/probes/fwd_scaling.py   (on the GPU box)
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us


def main():
    dev = torch.device("cuda:0")
    P = bench.pkg()
    sc = bench.Room0Scene(dev, 0, path="fused")
    eng = sc.engine
    ro, rd, gd, gc = sc.sample_batch()
    z = P.ops.sample_z(ro, rd, gd, sc.bound, 32, 16)
    for mult in (1, 2, 4, 8, 16):
        r_o, r_d, zz = ro.repeat(mult, 1), rd.repeat(mult, 1), z.repeat(mult, 1)
        n = zz.numel()
        row = []
        for stage in ("middle", "fine", "color"):
            for split in (False, True):
                P.ops.SPLIT_FWD = split
                us = timed(lambda: eng.query_fwd(stage, r_o, r_d, zz))
                row.append(f"{stage[:3]}{'/s' if split else '/f'} {us:7.1f}us ({us / n * 1e3:5.2f} ns/pt)")
        print(f"N={n:7d}  " + "  ".join(row), flush=True)
    P.ops.SPLIT_FWD = True
    # backward kernels per decoder, sequential, at 1x
    g_raw = torch.randn(z.numel(), 4, device=dev)
    eng.query_fwd("color", ro, rd, z)
    keys, dn = eng.grads_for("color", ("color",))
    for conc in (False, True):
        us = timed(lambda: eng.query_bwd("color", ro, rd, z, g_raw, keys, dn, concurrent=conc))
        print(f"query_bwd colour stage concurrent={conc}: {us:.1f} us", flush=True)


if __name__ == "__main__":
    main()
