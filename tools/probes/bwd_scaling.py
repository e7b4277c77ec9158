"""Backward time per decoder vs batch size (sequential launches), room0 colour-stage mapping.

python tools/probes/bwd_scaling.py   (on the GPU box)
"""
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from fwd_scaling import timed  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    P = bench.pkg()
    L = P._lib.lib()
    sc = bench.Room0Scene(dev, 0, path="fused")
    eng = sc.engine
    ro, rd, gd, gc = sc.sample_batch()
    z = P.ops.sample_z(ro, rd, gd, sc.bound, 32, 16)
    for mult in (1, 2, 4, 8):
        r_o, r_d, zz = ro.repeat(mult, 1), rd.repeat(mult, 1), z.repeat(mult, 1)
        n = zz.numel()
        g_raw = torch.randn(n, 4, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
        eng.query_fwd("color", r_o, r_d, zz)
        keys, dn = eng.grads_for("color", ("color",))
        cfg = eng._cfg("color", r_o, r_d, zz, keys, dn)
        row = []
        for name, d in (("mid", 1), ("fine", 2), ("col", 3)):
            wsb = L.nslam_query_bwd_decoder_workspace_size(ctypes.byref(cfg), d, n)
            ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
            st = torch.cuda.current_stream().cuda_stream

            def run():
                rc = L.nslam_query_bwd_decoder(ctypes.byref(cfg), d, 0, None, n, g_raw.data_ptr(), None,
                                               ws.data_ptr() if wsb else None, wsb, st)
                assert rc == 0, rc
            us = timed(run)
            row.append(f"{name} {us:7.1f}us ({us / n * 1e3:5.2f} ns/pt)")
        us = timed(lambda: eng.query_bwd("color", r_o, r_d, zz, g_raw, keys, dn, concurrent=True))
        row.append(f"all-concurrent {us:7.1f}us ({us / n * 1e3:5.2f} ns/pt)")
        print(f"N={n:7d}  " + "  ".join(row), flush=True)


if __name__ == "__main__":
    main()
