"""Tracking-iteration probe: 30 eager TrackingEngine iterations at room0 shape (200 pixels × 48),
for `rocprofv3 --kernel-trace --stats` (which kernels make up the 0.59 ms iteration)."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402

P = bench.pkg()
dev = torch.device("cuda:0")
scene = bench.Room0Scene(dev, 0, cfg=dict(bench.ROOM0))
cfg = scene.cfg
te = P.engine.TrackingEngine(copy.deepcopy(scene.nice), scene.grids, scene.bound, cfg["n_strat"], cfg["n_surf"],
                             (cfg["H"], cfg["W"]), (cfg["fx"], cfg["fy"], cfg["cx"], cfg["cy"]), ignore_edge=(100, 100),
                             device=dev)
cam = P.common.get_tensor_from_camera(scene.c2w[0]).to(dev).requires_grad_(True)
opt = P.ops.FusedAdam([{"params": [cam], "lr": 0.001}])
nwin = te.n_window()
for it in range(40):
    if it == 10:
        torch.cuda.synchronize()
        torch.cuda.nvtx.range_push("timed") if hasattr(torch.cuda, "nvtx") else None
    pix = torch.randint(nwin, (200,), device=dev)
    te.iteration(cam, scene.depth[0], scene.color[0], pix, opt)
torch.cuda.synchronize()
print("done")
