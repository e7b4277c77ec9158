"""Mapping-iteration time under engine knobs (one process, hipGraph-replayed like bench.py).

python tools/probes/knobs.py [knob names]   (NSLAM_FWD_PARTS, NSLAM_LIB are per-process)
Prints ms/iteration and M ray-samples/s for: the default engine, the weight-gradient branch on a
high-priority stream, and sequential (non-concurrent) decoder backward launches.
"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def timed(scene, steps=200):
    for _ in range(5):
        scene.step()
    torch.cuda.synchronize()
    g, _ = bench.capture_step_graphs(scene.step, sync=scene.flip_parity)
    g.run(g.block)
    torch.cuda.synchronize()
    scene.kept.zero_()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.run(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    g.finish()
    samples = int(scene.kept) * (scene.cfg["n_strat"] + scene.cfg["n_surf"])
    return dt / steps * 1e3, samples / dt / 1e6


def main():
    dev = torch.device("cuda:0")
    scene = bench.Room0Scene(dev, 0, path="fused")
    tag = os.environ.get("NSLAM_FWD_PARTS", "auto") + " " + os.path.basename(os.environ.get("NSLAM_LIB", "libnslam.so"))
    base = {"priority": False, "concurrent": True, "all_side": False, "lean_first": False, "merge_frozen": True,
            "split_wgrad": False, "wgrad_side": True}
    for name, knobs in (("default", {}), ("priority", {"priority": True}), ("sequential", {"concurrent": False}),
                        ("all_side", {"all_side": True}), ("lean_first", {"lean_first": True}),
                        ("side+lean", {"all_side": True, "lean_first": True}), ("merged", {"merge_frozen": True}), ("merged_all", {"merge_frozen": "all"}),
                        ("merged+prio", {"merge_frozen": True, "priority": True}),
                        ("merged+side", {"merge_frozen": True, "all_side": True}),
                        ("merged+lean_first", {"merge_frozen": True, "lean_first": True}),
                        ("unmerged", {"merge_frozen": False}),
                        ("split", {"split_wgrad": True}), ("split_main", {"split_wgrad": True, "wgrad_side": False}),
                        ("default", {})):
        if len(sys.argv) > 1 and name not in sys.argv[1:]:
            continue
        knobs = {**base, **knobs}
        for k, v in knobs.items():
            setattr(scene.engine, k, v)
        ms, rate = timed(scene)
        print(f"parts={tag} {name:10s} {ms:.4f} ms/iter  {rate:.2f} M ray-samples/s", flush=True)


if __name__ == "__main__":
    main()
