"""Cycle marks of k_color_wgrad (phases build): per wave role, the median cycles of each step of
the chunk's third tile, and the kernel's start/end spread.

NSLAM_LIB=nice-slam_amd/libnslam_phases.so python tools/probes/cw_phases.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
os.environ.setdefault("NSLAM_LIB", os.path.join(REPO, "nice-slam_amd", "libnslam_phases.so"))
import bench  # noqa: E402

STEPS = {(1, 2): "LDS-DMA issue", (2, 3): "compute", (3, 4): "end barrier"}


def main():
    dev = torch.device("cuda:0")
    P = bench.pkg()
    scene = bench.Room0Scene(dev, 0, path="fused")
    scene.engine.concurrent = "--concurrent" in sys.argv
    for _ in range(4):
        scene.step()
    torch.cuda.synchronize()
    L = P._lib.lib()
    L.nslam_debug_phases.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    W = 1 << 15
    buf = np.zeros(4 * W * 16, dtype=np.uint64)
    assert L.nslam_debug_phases(buf.ctypes.data, buf.size) == 0
    t = buf.reshape(4, W, 16).astype(np.int64)[0, 16384:]
    used = t[:, 0] != 0
    nw = int(used.sum())
    t = t[:nw]
    print(f"k_color_wgrad: {nw // 8} chunks")
    t0 = t[:, 0].min()
    print("  start p0/p50/max", *(np.percentile(t[:, 0] - t0, q).round() for q in (0, 50, 100)),
          "| end(pre-store) p50/p90/max", *(np.percentile(t[:, 8] - t0, q).round() for q in (50, 90, 100)))
    tot = t[:, 8] - t[:, 0]
    print(f"  wave loop cycles median {np.median(tot):.0f}")
    third = t[:, 1] != 0
    role = np.arange(nw) % 8
    for w in range(8):
        sel = third & (role == w)
        tt = t[sel]
        if not len(tt):
            continue
        parts = " ".join(f"{nm} {np.median(tt[:, b] - tt[:, a]):6.0f}" for (a, b), nm in STEPS.items()
                         if (tt[:, a] != 0).all() and (tt[:, b] != 0).all())
        print(f"  wave {w}: tile {np.median(tt[:, 4] - tt[:, 1]):6.0f} | {parts}")


if __name__ == "__main__":
    main()
