"""Mapping-iteration time (hipGraph replay) under engine variants: sequential / concurrent decoder
backward, with or without a high-priority stream for the weight-gradient branch.

python tools/probes/step_variants.py   (on the GPU box)
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402


SCENE = None


def graph_ms(fn, reps=100):
    for _ in range(3):
        fn()
    g, _ = bench.capture_step_graphs(fn, sync=SCENE.flip_parity)
    g.run(g.block)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.run(reps)
    b.record()
    torch.cuda.synchronize()
    g.finish()
    return a.elapsed_time(b) / reps * 1e3


def main():
    dev = torch.device("cuda:0")
    P = bench.pkg()
    sc = bench.Room0Scene(dev, 0, path="fused")
    global SCENE
    SCENE = sc
    eng = sc.engine
    variants = [("sequential", False, False), ("concurrent", True, False), ("concurrent+priority", True, True)]
    for rnd in range(2):
        for name, conc, prio in variants:
            eng.concurrent, eng.priority = conc, prio
            us = graph_ms(lambda: sc.step())
            P.ops.TIMER = P.ops.KernelTimer()
            for _ in range(20):
                sc.step()
            t = P.ops.TIMER.summary()
            P.ops.TIMER = None
            ks = " ".join(f"{k}={v['avg_ms'] * 1e3:.0f}" for k, v in t.items() if k.startswith("query_bwd"))
            print(f"[{rnd}] {name:22s} step {us:7.1f} us   eager: {ks}", flush=True)


if __name__ == "__main__":
    main()
