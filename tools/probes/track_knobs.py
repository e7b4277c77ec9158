"""Tracking-iteration time (hipGraph-replayed, room0 shape: 200 pixels x 48 samples) under engine
knobs, A/B in one process: merged frozen-decoder backward with the in-kernel d/dpts sum, merged with
per-decoder buffers added in torch, and one launch per decoder on separate streams.

python tools/probes/track_knobs.py
"""
import copy
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main(reps=300):
    P = bench.pkg()
    dev = torch.device("cuda:0")
    scene = bench.Room0Scene(dev, 0, path="fused")
    cfg = scene.cfg
    te = P.engine.TrackingEngine(copy.deepcopy(scene.nice), scene.grids, scene.bound, cfg["n_strat"], cfg["n_surf"],
                                 (cfg["H"], cfg["W"]), (cfg["fx"], cfg["fy"], cfg["cx"], cfg["cy"]),
                                 ignore_edge=(100, 100), w_color=0.5, handle_dynamic=True, use_color=True, device=dev)
    cam = P.common.get_tensor_from_camera(scene.c2w[0]).to(dev).requires_grad_(True)
    opt = P.ops.FusedAdam([{"params": [cam], "lr": 0.001}])
    nwin = te.n_window()

    def track():
        pix = torch.randint(nwin, (200,), device=dev)
        te.iteration(cam, scene.depth[0], scene.color[0], pix, opt)

    configs = (("sum", None, True), ("nosum", None, False), ("separate", False, True))
    for rnd in range(2):
        for name, merge, sum_pts in configs:
            te.eng.merge_frozen, te.eng.sum_pts = merge, sum_pts
            for _ in range(3):
                track()
            torch.cuda.synchronize()
            g, _ = bench.capture_step_graphs(track)
            g.run(20)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.run(reps)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / reps * 1e3
            print(f"round {rnd} {name:9s} {ms:.4f} ms/tracking iteration", flush=True)


if __name__ == "__main__":
    main()
