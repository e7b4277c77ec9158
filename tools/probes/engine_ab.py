"""In-process A/B of MappingEngine knobs on the room0 colour-stage bench iteration (hipGraph blocks,
as bench.py times them): alternating rounds, median ms per iteration per setting.

python tools/probes/engine_ab.py [rounds] [reps]
"""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402

SETTINGS = {  # engine attributes, or "bench.X" for bench.py module knobs
    "default": {},
    "no_prefetch": {"bench.PREFETCH": False},
    "lean_first": {"wgrad_first": False},
    "serial": {"concurrent": False},
}


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    dev = torch.device("cuda:0")
    scene = bench.Room0Scene(dev, 0, path="fused")
    eng = scene.engine
    def owner(k):
        return (bench, k[6:]) if k.startswith("bench.") else (eng, k)

    base = {k: getattr(*owner(k)) for s in SETTINGS.values() for k in s}
    res = {k: [] for k in SETTINGS}
    for r in range(rounds):
        for name, knobs in SETTINGS.items():
            for k, v in base.items():
                setattr(*owner(k), v)
            for k, v in knobs.items():
                setattr(*owner(k), v)
            ms, mode = bench.graph_time(scene, scene.step, reps)
            res[name].append(ms)
            print(f"round {r} {name:12s} {ms:.4f} ms ({mode})", flush=True)
    for name, v in res.items():
        med = statistics.median(v)
        print(f"{name:12s} median {med:.4f} ms  {48000 / med / 1e3:.1f} M ray-samples/s (nominal 48k)  all {[round(x, 4) for x in v]}")


if __name__ == "__main__":
    main()
