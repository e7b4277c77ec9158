"""Tracker probe: Tracker.track_frame (one captured hipGraph per frame) at room0 shape as the SLAM-loop leg
runs it (10 camera iterations x 200 pixels, edges 100 px), 40 frames after 10 warm-up ones, no mapping; prints
the wall time per frame.  Run under `rocprofv3 --kernel-trace --stats` to see one frame's kernels."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402

P = bench.pkg()
dev = torch.device("cuda:0")
scene = bench.Room0Scene(dev, 0, cfg=dict(bench.ROOM0), path="autograd")
for t in scene.grids.values():
    t.requires_grad_(False)
tr = P.Tracker(bench.nice_slam_cfg(bench.ROOM0), None, bench.slam_state(scene))
nudge = torch.tensor([0.02, -0.01, 0.015], device=dev)


def frame(i):
    f = i % bench.ROOM0["window"]
    gt = bench._pose4(scene.c2w[f])
    pre = gt.clone()
    pre[:3, 3] += nudge
    return tr.track_frame(i + 1, scene.color[f], scene.depth[f], gt, pre_c2w=pre)


for i in range(10):
    frame(i)
torch.cuda.synchronize()
n = 40
t0 = time.perf_counter()
for i in range(10, 10 + n):
    frame(i)
torch.cuda.synchronize()
print(f"track_frame {(time.perf_counter() - t0) / n * 1e3:.3f} ms per frame (async, {n} frames)")
ts = []
for i in range(10 + n, 20 + n):
    t0 = time.perf_counter()
    frame(i)
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e3)
print(f"track_frame {sum(ts) / len(ts):.3f} ms per frame (synchronised)")
