"""Per-phase cycle breakdown of the backward tile (instrumented build, make -C nice-slam_amd/csrc phases).

NSLAM_LIB=nice-slam_amd/libnslam_phases.so python tools/probes/phases.py
Runs room0 colour-stage mapping iterations with sequential decoder launches and prints, per
decoder kernel, the distribution over waves of the cycles between consecutive s_memtime marks.
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

NAMES = {0: "start", 1: "point+g", 2: "corners", 3: "gather", 4: "fwd recompute", 5: "out layer(+dWo)",
         6: "layer4", 7: "layer3", 8: "layer2", 9: "layer1", 10: "layer0", 11: "fourier", 12: "pre-scatter",
         13: "scatter", 14: "end"}


def main():
    dev = torch.device("cuda:0")
    P = bench.pkg()
    scene = bench.Room0Scene(dev, 0, path="fused")
    scene.engine.concurrent = False
    scene.engine.merge = False  # one kernel per decoder: wave index = tile in every phase slot
    for _ in range(4):
        scene.step()
    torch.cuda.synchronize()
    L = P._lib.lib()
    L.nslam_debug_phases.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    W = 1 << 15
    buf = np.zeros(5 * W * 16, dtype=np.uint64)
    assert L.nslam_debug_phases(buf.ctypes.data, buf.size) == 0
    buf = buf.reshape(5, W, 16).astype(np.int64)
    tiles = (scene.cfg["pixels"] * 48 + 31) // 32
    fwd_names = {0: "start", 1: "point", 2: "corners", 3: "gather", 5: "emb+L0+L3e", 6: "L1+L2", 7: "L3", 8: "L4",
                 9: "out+store", 10: "c.corners", 11: "c.gather", 12: "c.emb+L0+L3e", 13: "c.L1+L2", 14: "c.L3",
                 15: "c.L4"}
    print("nonzero marks per slot:", [int((buf[k] != 0).sum()) for k in range(5)])
    # room0 colour stage: the 2-part forward (middle then colour | fine), parts alternating along
    # blockIdx (k_query_fwd_parts); 4 waves per workgroup
    groups = (tiles + 3) // 4
    nw = groups * 2 * 4
    t = buf[0, :nw]
    part = (np.arange(nw) // 4) % 2
    for pi, nm in ((0, "middle then colour"), (1, "fine")):
        tp = t[(part == pi) & (t[:, 0] != 0)]
        marks = [k for k in range(16) if (tp[:, k] != 0).all()]
        marks.sort(key=lambda k: np.median(tp[:, k] - tp[:, 0]))  # in time order (part 0: middle, then colour)
        tot = tp[:, marks[-1]] - tp[:, marks[0]]
        print(f"== forward part {nm}: {len(tp)} waves, marks {marks}; wave total median {np.median(tot):.0f} "
              f"p10 {np.percentile(tot, 10):.0f} p90 {np.percentile(tot, 90):.0f}")
        t0 = np.percentile(t[t[:, 0] != 0][:, 0], 0.5)  # robust to stale marks
        st, en = tp[:, marks[0]] - t0, tp[:, marks[-1]] - t0
        print("   start offsets p0/p50/p90/p99/max " + " ".join(f"{np.percentile(st, q):.0f}" for q in (0, 50, 90, 99, 100))
              + " | end p50/p90/max " + " ".join(f"{np.percentile(en, q):.0f}" for q in (50, 90, 100)))
        for a_, b_ in zip(marks[:-1], marks[1:]):
            dt = tp[:, b_] - tp[:, a_]
            print(f"   {fwd_names[a_]:>12s} -> {fwd_names[b_]:<12s} median {np.median(dt):8.0f}  "
                  f"({100 * np.median(dt) / max(np.median(tot), 1):5.1f}%)")
    # k_color_wgrad: per wave (8 per workgroup, one chunk of tiles each) the cycles producing the next
    # tile, consuming this one and waiting at the hand-over barriers
    cw = buf[4]
    nwg = int((cw[:, 3] > 0).sum()) // 8
    if nwg:
        cw = cw[:nwg * 8].reshape(nwg, 8, 16)
        roles = {0: "S_b dW3/dW0", 1: "S_b dW3/dW0", 2: "S_b dW3/dW0", 3: "feature+h2/dW2",
                 4: "fc_c+dB", 5: "fc_c+dB", 6: "fc_c.2,dW4+dB", 7: "chain producer"}
        perm = [(0x52104637 >> (4 * w)) & 15 for w in range(8)]  # k_color_wgrad's role of hardware wave w
        print(f"== k_color_wgrad: {nwg} workgroups, tiles per chunk median {np.median(cw[:, 0, 3]):.0f}")
        for wv in range(8):
            tp, tc, th = (np.median(cw[:, wv, k]) for k in range(3))
            tot = tp + tc + th
            print(f"   hw wave {wv} (SIMD {wv % 4}) role {perm[wv]} {roles[perm[wv]]:>16s}: prod {tp:8.0f}  "
                  f"cons {tc:8.0f}  wait {th:8.0f}  (wait {100 * th / max(tot, 1):5.1f}%)")
    for d, nm in ((1, "middle"), (2, "fine"), (3, "color")):
        t = buf[d, :tiles]
        marks = [k for k in range(16) if (t[:, k] != 0).all()]
        print(f"== {nm} decoder backward: {tiles} waves, marks {marks}")
        tot = t[:, marks[-1]] - t[:, marks[0]]
        st = t[:, marks[0]] - t[:, marks[0]].min()
        print(f"   wave total cycles: median {np.median(tot):.0f}  p10 {np.percentile(tot, 10):.0f}  "
              f"p90 {np.percentile(tot, 90):.0f};  start spread p50 {np.median(st):.0f} max {st.max():.0f}; "
              f"kernel span {(t[:, marks[-1]].max() - t[:, marks[0]].min()):.0f}")
        for a, b in zip(marks[:-1], marks[1:]):
            dt = t[:, b] - t[:, a]
            print(f"   {NAMES[a]:>16s} -> {NAMES[b]:<16s} median {np.median(dt):8.0f}  mean {dt.mean():8.0f}  "
                  f"({100 * np.median(dt) / max(np.median(tot), 1):5.1f}%)")


if __name__ == "__main__":
    main()
