"""Repeat the bench's graph-captured pieces in one process to localise an intermittent host-heap
corruption (run with MALLOC_CHECK_=3).  usage: python tools/probes/heap_probe.py [what] [n]"""
import copy
import faulthandler
import os
import sys
import time

faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402

what = sys.argv[1] if len(sys.argv) > 1 else "all"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 6
dev = torch.device("cuda:0")
scene = bench.Room0Scene(dev)
for _ in range(3):
    scene.step()
torch.cuda.synchronize()
for i in range(n):
    t0 = time.time()
    if what in ("all", "map"):
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            scene.step()
        torch.cuda.current_stream().wait_stream(side)
        with torch.cuda.graph(g):
            scene.step()
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        print(i, "map graph ok", flush=True)
    if what in ("all", "copy"):
        for _ in range(20):
            copy.deepcopy(scene.nice)
        print(i, "deepcopy ok", flush=True)
    if what in ("all", "frames"):
        r = bench.room0_frame_rate(scene, reps=5)
        print(i, "frames ok", r["frames_per_s"], flush=True)
    print(i, "iteration", round(time.time() - t0, 2), "s", flush=True)
print("PROBE DONE", flush=True)
