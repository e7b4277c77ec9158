"""Per-wave timeline of the mapping iteration's big kernels (timeline build: make -C nice-slam_amd/csrc timeline).

NSLAM_LIB=nice-slam_amd/libnslam_tl.so python tools/probes/wave_timeline.py [--no-prefetch] [--serial]
Every wave of k_query_fwd_parts (slot 0), k_dec_bwd_multi (slot 1) and k_color_wgrad (slot 2) records
s_memrealtime (100 MHz, one clock for every XCD) at its start and end, and its HW_ID / XCC_ID.  Prints,
per kernel of the last iteration: the span, when waves start (dispatch), their lifetimes, the waves each
SIMD received and how many were resident at once, and the mean resident waves per SIMD over the span.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
os.environ.setdefault("NSLAM_LIB", os.path.join(REPO, "nice-slam_amd", "libnslam_tl.so"))
import bench  # noqa: E402

W = 1 << 15
TICK_US = 0.01  # s_memrealtime: 100 MHz


def analyse(name, t, parts=None):
    ok = (t[:, 0] != 0) & (t[:, 1] >= t[:, 0])
    t = t[ok]
    if not len(t):
        print(f"== {name}: no waves")
        return
    st, en, hw = t[:, 0], t[:, 1], t[:, 2]
    t0 = st.min()
    simd = ((hw >> 4) & 3) | (((hw >> 8) & 15) << 2) | (((hw >> 12) & 1) << 6) | (((hw >> 13) & 7) << 7) | \
        (((hw >> 32) & 15) << 10)
    cu = simd >> 2
    span = (en.max() - t0) * TICK_US
    life = (en - st) * TICK_US
    print(f"== {name}: {len(t)} waves, span {span:.1f} us, {len(np.unique(simd))} SIMDs, {len(np.unique(cu))} CUs")
    q = (0, 10, 50, 90, 99, 100)
    print("   start (us after the first)  " + " ".join(f"p{p}={np.percentile((st - t0) * TICK_US, p):.1f}" for p in q))
    print("   end                         " + " ".join(f"p{p}={np.percentile((en - t0) * TICK_US, p):.1f}" for p in q))
    print("   lifetime                    " + " ".join(f"p{p}={np.percentile(life, p):.1f}" for p in q))
    if parts is not None:
        waits = ((parts[ok] >> 8) & 0xffffff) * TICK_US  # time the wave spent polling flags (k_query_fwd_pc)
        field1 = ((parts[ok] >> 32) & 0xffffff) * TICK_US  # a second timed phase (the pc producer's gathers)
        parts = parts & 0xff
        pp = parts[ok]
        for v in np.unique(pp):
            lv = life[pp == v]
            wv = waits[pp == v]
            extra = f", waiting {wv.mean():.1f} us ({wv.sum() / lv.sum():.0%})" if wv.any() else ""
            f1 = field1[pp == v]
            extra += f", gathering {f1.mean():.1f} us ({f1.sum() / lv.sum():.0%})" if f1.any() else ""
            print(f"     part {v}: {len(lv)} waves, lifetime p50 {np.median(lv):.1f} p90 {np.percentile(lv, 90):.1f}"
                  f" mean {lv.mean():.1f} us{extra}")
    # per SIMD: waves received, max resident at once, busy span (first start .. last end)
    us, inv = np.unique(simd, return_inverse=True)
    cnt = np.bincount(inv)
    if parts is not None:  # which tags (parts / roles) share a SIMD: "tag0 x tag1 x ..." -> SIMDs
        pp = parts[ok]
        tags = np.unique(pp)
        combo = {}
        for i in range(len(us)):
            key = " ".join(f"{int((pp[inv == i] == v).sum())}" for v in tags)
            combo[key] = combo.get(key, 0) + 1
        print(f"   waves of tags {list(map(int, tags))} per SIMD: " +
              ", ".join(f"[{k}]:{v}" for k, v in sorted(combo.items(), key=lambda e: -e[1])[:6]))
    print("   waves per SIMD: " + ", ".join(f"{k}:{v}" for k, v in zip(*np.unique(cnt, return_counts=True))))
    maxres, last_end = [], []
    for i in range(len(us)):
        sel = inv == i
        ev = sorted([(a, 1) for a in st[sel]] + [(b, -1) for b in en[sel]], key=lambda e: (e[0], e[1]))
        c = m = 0
        for _, d in ev:
            c += d
            m = max(m, c)
        maxres.append(m)
        last_end.append((en[sel].max() - t0) * TICK_US)
    print("   max resident per SIMD: " + ", ".join(f"{k}:{v}" for k, v in zip(*np.unique(maxres, return_counts=True))))
    le = np.array(last_end)
    print("   SIMD last wave ends (us)    " + " ".join(f"p{p}={np.percentile(le, p):.1f}" for p in q))
    nsimd = 1024
    print(f"   mean resident waves per SIMD over the span: {life.sum() / (span * nsimd):.2f} "
          f"(over SIMDs that ran waves: {life.sum() / (span * len(us)):.2f})")
    # resident-wave histogram over time (chip total), 10 bins
    edges = np.linspace(0, span, 11)
    res = []
    for a, b in zip(edges[:-1], edges[1:]):
        lo, hi = t0 + a / TICK_US, t0 + b / TICK_US
        ov = np.clip(np.minimum(en, hi) - np.maximum(st, lo), 0, None).sum() * TICK_US
        res.append(ov / ((b - a) * nsimd))
    print("   resident waves/SIMD by tenth of the span: " + " ".join(f"{r:.2f}" for r in res))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-prefetch", action="store_true")
    ap.add_argument("--serial", action="store_true", help="branches serialised (no concurrent kernels)")
    ap.add_argument("--iters", type=int, default=6)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    P = bench.pkg()
    scene = bench.Room0Scene(dev, 0, path="fused")
    if args.serial:
        scene.engine.concurrent = False
    if args.no_prefetch:
        bench.PREFETCH = False
    for _ in range(args.iters):
        scene.step()
    torch.cuda.synchronize()
    L = P._lib.lib()
    L.nslam_debug_timeline.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    buf = np.zeros(3 * W * 4, dtype=np.uint64)
    assert L.nslam_debug_timeline(buf.ctypes.data, buf.size) == 0
    buf = buf.reshape(3, W, 4).astype(np.int64)
    print(f"mode: prefetch={not args.no_prefetch} serial={args.serial}")
    analyse("k_query_fwd_parts", buf[0], parts=buf[0][:, 3])
    analyse("k_dec_bwd_multi", buf[1], parts=buf[1][:, 3])
    analyse("k_color_wgrad", buf[2])
    # overlap of the three kernels of the last iteration
    rng = []
    for k in range(3):
        t = buf[k][(buf[k][:, 0] != 0)]
        if len(t):
            rng.append((t[:, 0].min(), t[:, 1].max()))
    if rng:
        base = min(r[0] for r in rng)
        print("kernel windows (us): " + ", ".join(f"[{(a - base) * TICK_US:.1f}, {(b - base) * TICK_US:.1f}]"
                                             for a, b in rng))


if __name__ == "__main__":
    main()
