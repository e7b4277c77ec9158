"""CPU-side checks of the boundary: libnslam.so loads, exports every symbol include/nslam.h
declares, and the Python pack layout agrees with the C++ one (no GPU calls)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import REPO


def _header_symbols():
    txt = open(os.path.join(REPO, "include", "nslam.h")).read()
    return sorted(set(re.findall(r"\b(nslam_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_header_symbol(pkg):
    L = pkg._lib.lib()
    syms = _header_symbols()
    assert len(syms) >= 10
    for name in syms:
        assert hasattr(L, name), f"libnslam.so does not export {name}"
    assert set(syms) == set(pkg._lib.EXPORTS)


def test_abi_version_and_strerror(pkg):
    L = pkg._lib.lib()
    assert L.nslam_abi_version() == pkg._lib.ABI_VERSION == 23
    assert L.nslam_strerror(0) == b"ok"
    assert b"invalid" in L.nslam_strerror(-1)


def test_pack_layout_matches_python(pkg):
    P = pkg.packing
    for nc in (1, 2):
        c = pkg._lib.pack_layout(0, nc)
        py = P.xyz_layout(nc)
        assert c["total"] == py["total"] and c["vec"] == py["V"]
        assert c["nf"] == py["nf"] and c["nb"] == py["nfrag"] - py["nf"]
    c = pkg._lib.pack_layout(1, 1)
    py = P.noxyz_layout()
    assert c["total"] == py["total"] and c["vec"] == py["V"] and c["nf"] == py["nf"]


def test_argument_validation_without_gpu(pkg):
    """Entry points reject bad arguments before touching the device."""
    L = pkg._lib.lib()
    cfg = pkg._lib.NslamQueryCfg()
    cfg.stage = 7
    assert L.nslam_query_fwd(ctypes.byref(cfg), None, 10, None, None) == -1
    assert L.nslam_query_bwd(ctypes.byref(cfg), None, 10, None, None, None, 0, None) == -1
    assert L.nslam_composite_fwd(None, None, 4, 0, None, None, None, None) == -1
    assert L.nslam_composite_fwd(None, None, 4, 1000, None, None, None, None) == -2
    dims = (ctypes.c_int32 * 3)(0, 1, 1)
    assert L.nslam_grid_sample_fwd(None, dims, None, 5, None, None) == -1
    lo = (ctypes.c_double * 3)(0, 0, 0)
    assert L.nslam_sample_rays(None, None, None, None, 3, lo, lo, None, 500, None, 0, 0, None, None, 0, None) == -2
    assert L.nslam_rows_pack(None, None, 4, 30, None, 0, None, None) == -1      # row_len % 4
    assert L.nslam_rows_pack(None, None, 4, 32, None, 0, None, None) == -1      # NULL grid/rows
    assert L.nslam_rows_unpack(None, None, 0, 32, None, None, 5, None) == -1    # NULL tail
    assert L.nslam_rows_pack(None, None, 0, 32, None, 0, None, None) == 0       # empty: no launch


def test_no_cpu_fallback(pkg):
    import torch
    with pytest.raises(RuntimeError, match="HIP device"):
        pkg.ops.composite(torch.zeros(2, 4, 4), torch.zeros(2, 4, dtype=torch.float64))


def test_struct_layouts_match_header(pkg, tmp_path):
    """sizeof/offsetof of every ABI struct, compiled by gcc from include/nslam.h, equal the ctypes
    mirrors in _lib.py."""
    L = pkg._lib
    structs = {"nslam_grid": L.NslamGrid, "nslam_dec_grad": L.NslamDecGrad, "nslam_query_cfg": L.NslamQueryCfg,
               "nslam_frame": L.NslamFrame, "nslam_loss_cfg": L.NslamLossCfg, "nslam_adam_seg": L.NslamAdamSeg,
               "nslam_draw": L.NslamDraw}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "nslam.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for f in py._fields_:
            lines.append(f'  printf("{cname} {f[0]} %zu\\n", offsetof({cname}, {f[0]}));')
    lines.append("  return 0; }")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {tuple(l.split()[:2]): int(l.split()[2]) for l in out if l}
    for cname, py in structs.items():
        assert got[(cname, "size")] == ctypes.sizeof(py), cname
        for f in py._fields_:
            assert got[(cname, f[0])] == getattr(py, f[0]).offset, (cname, f[0])


def test_v4_entry_points_validate_without_gpu(pkg):
    L = pkg._lib.lib()
    lib = pkg._lib
    fr = (lib.NslamFrame * 1)()
    assert L.nslam_gather_rays(fr, 0, 10, None, 10, 10, 0, 10, 0, 10, 1.0, 1.0, 0.0, 0.0, None, None,
                               None, None, None, None, None, None, None, None) == -1
    assert L.nslam_gather_rays(fr, 1, 10, None, 10, 10, 0, 11, 0, 10, 1.0, 1.0, 0.0, 0.0, None, None,
                               None, None, None, None, None, None, None, None) == -1
    # ABI v7: neither pix nor draws, and draws without device counter/ticket, are rejected
    fr[0].depth = fr[0].color = fr[0].c2w = 64
    assert L.nslam_gather_rays(fr, 1, 10, None, 10, 10, 0, 10, 0, 10, 1.0, 1.0, 0.0, 0.0, None, None,
                               64, 64, 64, 64, None, None, None, None) == -1
    draw = lib.NslamDraw(7, None, None)
    assert L.nslam_gather_rays(fr, 1, 10, None, 10, 10, 0, 10, 0, 10, 1.0, 1.0, 0.0, 0.0, None, None,
                               64, 64, 64, 64, None, ctypes.byref(draw), None, None) == -1
    cfg = lib.NslamLossCfg(5, 0, 0, 0.2)
    assert L.nslam_render_loss(ctypes.byref(cfg), None, None, 4, 48, None, None, None, None, None, None, None,
                               None, None, 0, None) == -1
    cfg = lib.NslamLossCfg(lib.LOSS_MAPPER, 0, 0, 0.2)
    assert L.nslam_render_loss(ctypes.byref(cfg), None, None, 4, 1000, None, None, None, None, None, None, None,
                               None, None, 0, None) == -2
    cfg = lib.NslamLossCfg(lib.LOSS_TRACKER, 1, 1, 0.5)
    assert L.nslam_render_loss_workspace_size(ctypes.byref(cfg), 100) == 101 * 8
    seg = (lib.NslamAdamSeg * 1)()
    assert L.nslam_adam_step(seg, 0, 0.9, 0.999, 1e-8, 1, None, None) == -1
    seg[0].n, seg[0].rows, seg[0].row_len = 4, 16, 6   # row_len % 4 != 0
    for f in ("param", "grad", "exp_avg", "exp_avg_sq", "step"):
        setattr(seg[0], f, 64)
    assert L.nslam_adam_step(seg, 1, 0.9, 0.999, 1e-8, 1, 64, None) == -1


def test_v8_cam_grad_validates_without_gpu(pkg):
    L = pkg._lib.lib()
    assert L.nslam_cam_grad(None, 64, 64, 64, 64, 10, 48, 64, None) == -1   # no cam
    assert L.nslam_cam_grad(64, 64, 64, 64, 64, -1, 48, 64, None) == -1     # negative ray count
    assert L.nslam_cam_grad(64, 64, None, 64, 64, 10, 48, 64, None) == -1   # rays without g_pts
    assert L.nslam_cam_grad(64, 64, 64, 64, 64, 10, 0, 64, None) == -1      # no samples
    # g_pts rows are indexed p*3+k in 32 bits: 3 * rays * samples must stay below 2^31
    assert L.nslam_cam_grad(64, 64, 64, 64, 64, (1 << 31) // 3 // 48 + 1, 48, 64, None) == -2


def test_v8_cam_pose_validates_without_gpu(pkg):
    L = pkg._lib.lib()
    assert L.nslam_cam_pose(None, 64, None) == -1
    assert L.nslam_cam_pose(64, None, None) == -1


def _colour_cfg(pkg):
    """A colour-stage config with fake (aligned, never dereferenced) device pointers: the entry points
    below must reject or accept it from the arguments alone, before any launch."""
    cfg = pkg._lib.NslamQueryCfg()
    cfg.stage = pkg._lib.STAGES["color"]
    for d in range(4):
        cfg.grid[d].data = 4096
        cfg.grid[d].dims[0] = cfg.grid[d].dims[1] = cfg.grid[d].dims[2] = 8
        cfg.packed[d] = 4096
    return cfg


def test_v16_bwd_decoders_validates_without_gpu(pkg):
    """nslam_query_bwd_decoders rejects bad configs, masks and parameter gradients before any launch."""
    L = pkg._lib.lib()
    cfg = pkg._lib.NslamQueryCfg()
    cfg.stage = 7
    gps = (ctypes.c_void_p * 4)()
    assert L.nslam_query_bwd_decoders(ctypes.byref(cfg), 0b0110, None, 10, None, gps, None) == -1  # stage
    ok = pkg._lib.NslamQueryCfg()
    rc = L.nslam_query_bwd_decoders(ctypes.byref(ok), 0, None, 0, None, gps, None)
    assert rc < 0  # an empty decoder mask (or an otherwise incomplete config) is never launched
    c = _colour_cfg(pkg)
    c.dgrad[pkg._lib.DEC_COLOR].base = 4096
    c.dgrad[pkg._lib.DEC_COLOR].count = 100
    colour = 1 << pkg._lib.DEC_COLOR
    # no parameter gradients in the lean launch (v16: the colour decoder's come from nslam_color_wgrad)
    assert L.nslam_query_bwd_decoders(ctypes.byref(c), colour, 4096, 10, 4096, gps, None) == -2
    c.dgrad[pkg._lib.DEC_COLOR].base = None
    assert L.nslam_query_bwd_decoders(ctypes.byref(c), colour, 4096, 10, 4096, gps, None) == -2  # no saved masks
    assert L.nslam_query_bwd_decoders(ctypes.byref(c), 1 << pkg._lib.DEC_COARSE, 4096, 10, 4096, gps, None) == -1


def test_v16_color_wgrad_validates_without_gpu(pkg):
    """nslam_color_wgrad rejects configs without a colour weight-gradient tape backward, a missing
    cotangent and a short workspace before any launch; an empty batch is a no-op."""
    L = pkg._lib.lib()
    cfg = pkg._lib.NslamQueryCfg()
    cfg.stage = 7
    assert L.nslam_color_wgrad(ctypes.byref(cfg), None, 10, None, None, 0, None) == -1            # bad stage
    c = _colour_cfg(pkg)
    c.stage = pkg._lib.STAGES["middle"]
    assert L.nslam_color_wgrad(ctypes.byref(c), 4096, 10, 4096, 4096, 1 << 20, None) == -1        # not colour
    c.stage = pkg._lib.STAGES["color"]
    assert L.nslam_color_wgrad(ctypes.byref(c), 4096, 10, 4096, 4096, 1 << 20, None) == -2        # no dgrad
    c.dgrad[pkg._lib.DEC_COLOR].base = 4096
    c.dgrad[pkg._lib.DEC_COLOR].count = 15575
    assert L.nslam_color_wgrad(ctypes.byref(c), 4096, 10, 4096, 4096, 1 << 20, None) == -2        # no tapes
    c.act_tape = 4096
    c.saved_masks = 4096
    assert L.nslam_color_wgrad(ctypes.byref(c), 4096, 10, None, 4096, 1 << 20, None) == -1        # no g_raw
    assert L.nslam_color_wgrad(ctypes.byref(c), None, 10, 4096, 4096, 1 << 20, None) == -1        # no points
    need = L.nslam_query_bwd_decoder_workspace_size(ctypes.byref(c), pkg._lib.DEC_COLOR, 10)
    assert need > 0
    assert L.nslam_color_wgrad(ctypes.byref(c), 4096, 10, 4096, 4096, need - 1, None) == -3       # short ws
    assert L.nslam_color_wgrad(ctypes.byref(c), 4096, 10, 4096, None, need, None) == -3           # no ws
    assert L.nslam_color_wgrad(ctypes.byref(c), None, 0, None, None, 0, None) == 0                # empty batch


def test_v16_removed_entry_points(pkg):
    """ABI v16 dropped the options measured neutral or slower in round 3 (the fused colour Adam, the
    part-wise forward of the pipelined loop): they are no longer exported."""
    L = pkg._lib.lib()
    for name in ("nslam_color_wgrad_adam", "nslam_query_fwd_parts"):
        assert not hasattr(L, name), name


def test_v15_cam_grad_parts_validates_without_gpu(pkg):
    """nslam_cam_grad_parts rejects missing buffers, bad part counts and oversized point counts."""
    L = pkg._lib.lib()
    bufs = (ctypes.c_void_p * 4)(64, 64, 64, 64)
    assert L.nslam_cam_grad_parts(64, 64, bufs, 3, 64, 64, 10, 48, 64, None, 64, None) == -1       # no ws
    assert L.nslam_cam_grad_parts(64, 64, bufs, 3, 64, 64, 10, 48, 64, 64, None, None) == -1       # no ticket
    assert L.nslam_cam_grad_parts(64, 64, bufs, 0, 64, 64, 10, 48, 64, 64, 64, None) == -1         # no parts
    assert L.nslam_cam_grad_parts(64, 64, bufs, 5, 64, 64, 10, 48, 64, 64, 64, None) == -1         # too many
    bufs[1] = None
    assert L.nslam_cam_grad_parts(64, 64, bufs, 3, 64, 64, 10, 48, 64, 64, 64, None) == -1         # a NULL part
    bufs[1] = 64
    assert L.nslam_cam_grad_parts(64, 64, bufs, 3, 64, 64, (1 << 31) // 3 // 48 + 1, 48, 64, 64, 64, None) == -2


def test_v19_cam_batch_validates_without_gpu(pkg):
    """nslam_cam_grad_batch / nslam_cam_pose_batch reject bad camera counts, strides, buffers and ray slices
    outside the batch before any launch."""
    L = pkg._lib.lib()
    bufs = (ctypes.c_void_p * 4)(64, 64, 64, 64)
    rb = (ctypes.c_int64 * 2)(0, 100)
    args = lambda **k: dict(dict(cams=64, c2w=64, stride=16, n=2, rb=rb, per=100, bufs=bufs, parts=3, z=64, rd=64,  # noqa: E731
                                 N=200, S=48, out=64, ws=64, tk=64), **k)

    def call(a):
        return L.nslam_cam_grad_batch(a["cams"], a["c2w"], a["stride"], a["n"], a["rb"], a["per"], a["bufs"],
                                      a["parts"], a["z"], a["rd"], a["N"], a["S"], a["out"], a["ws"], a["tk"], None)
    assert call(args(n=0)) == -1                       # no cameras
    assert call(args(n=33)) == -1                      # more than NSLAM_MAX_FRAMES
    assert call(args(stride=8)) == -1                  # a c2w stride shorter than a [3,4] pose
    assert call(args(tk=None)) == -1                   # no tickets
    assert call(args(ws=None)) == -1                   # no workspace
    assert call(args(parts=5)) == -1                   # too many d/dpts parts
    assert call(args(per=101)) == -1                   # camera 1's slice ends past the batch
    assert call(args(rb=None)) == -1                   # no slice table
    assert call(args(N=(1 << 31) // 3 // 48 + 1, per=100)) == -2
    assert L.nslam_cam_pose_batch(None, 64, 16, 2, None) == -1
    assert L.nslam_cam_pose_batch(64, 64, 16, 0, None) == -1
    assert L.nslam_cam_pose_batch(64, 64, 8, 2, None) == -1


def test_v20_frustum_rows_validates_without_gpu(pkg):
    L = pkg._lib.lib()
    need = L.nslam_frustum_rows_workspace_size(10 * 12 * 20)
    assert need > 2400 * 5 and L.nslam_frustum_rows_workspace_size(0) == 0
    args = [64, 64, 64, 680, 1200, 20, 12, 10, 64, 64, 64, None, 64, need, None]
    for i in (0, 1, 2, 8, 9, 10):  # a missing input / output buffer
        a = list(args)
        a[i] = None
        assert L.nslam_frustum_rows(*a) == -1, i
    a = list(args)
    a[5] = 0                            # an empty grid axis
    assert L.nslam_frustum_rows(*a) == -1
    a = list(args)
    a[13] = need - 1                    # short workspace
    assert L.nslam_frustum_rows(*a) == -3


def test_v21_loss_sum_best_validates_without_gpu(pkg):
    """nslam_loss_sum_best needs an output scalar (and a loss vector when there are rays); with a
    best_loss it needs the two camera vectors and 1 <= n <= 64 — all before any launch."""
    L = pkg._lib.lib()
    assert L.nslam_loss_sum_best(4096, 10, None, None, None, None, 0, None) == -1      # no output
    assert L.nslam_loss_sum_best(None, 10, 4096, None, None, None, 0, None) == -1      # no losses
    assert L.nslam_loss_sum_best(4096, -1, 4096, None, None, None, 0, None) == -1      # negative count
    assert L.nslam_loss_sum_best(4096, 10, 4096, 4096, None, 4096, 7, None) == -1     # best without cam
    assert L.nslam_loss_sum_best(4096, 10, 4096, 4096, 4096, 4096, 65, None) == -1    # n > 64


def test_v22_cam_vector_batch_validates_without_gpu(pkg):
    """nslam_cam_vector_batch needs poses and outputs, 1 <= n <= 64 and a pose stride of at least 12 floats
    — all checked before any launch (the copy is optional)."""
    L = pkg._lib.lib()
    assert L.nslam_cam_vector_batch(None, 16, 1, 4096, None, None) == -1     # no poses
    assert L.nslam_cam_vector_batch(4096, 16, 1, None, 4096, None) == -1     # no output
    assert L.nslam_cam_vector_batch(4096, 16, 0, 4096, None, None) == -1     # no cameras
    assert L.nslam_cam_vector_batch(4096, 16, 65, 4096, None, None) == -1    # n > 64
    assert L.nslam_cam_vector_batch(4096, 8, 2, 4096, None, None) == -1      # stride < 12


def test_v23_cam_grad_step_validates_without_gpu(pkg):
    """nslam_cam_grad_step needs its tail (camera, Adam state, step count, loss output; a loss vector when there
    are rays; the best pose with a best loss) before the gradient's own checks — all before any launch."""
    import ctypes
    L = pkg._lib.lib()
    T = pkg._lib.NslamCamTail
    bufs = (ctypes.c_void_p * 1)(4096)

    def call(tail):
        return L.nslam_cam_grad_step(None if tail is None else ctypes.byref(tail), 4096, bufs, 1, 4096, 4096, 10, 4,
                                     4096, 4096, 4096, None)

    def tail(**kw):
        f = dict(cam=4096, exp_avg=4096, exp_avg_sq=4096, step=4096, lr=0.001, beta1=0.9, beta2=0.999, eps=1e-8,
                 ray_loss=4096, n_rays=10, loss_out=4096, best_loss=None, best=None)
        f.update(kw)
        return T(**f)

    assert call(None) == -1
    assert call(tail(cam=None)) == -1
    assert call(tail(step=None)) == -1
    assert call(tail(loss_out=None)) == -1
    assert call(tail(ray_loss=None)) == -1
    assert call(tail(n_rays=-1)) == -1
    assert call(tail(best_loss=4096)) == -1            # best loss without the best pose
    assert L.nslam_cam_grad_step(ctypes.byref(tail()), None, bufs, 1, 4096, 4096, 10, 4, 4096, 4096, 4096,
                                 None) == -1           # the gradient's own checks (no pose)


def test_median_launch_knob_rejects_unknown_values(pkg, monkeypatch):
    """NSLAM_MEDIAN_LAUNCH accepts "0" and "1" only: any other value is NSLAM_EINVAL before any launch."""
    import ctypes
    L = pkg._lib.lib()
    cfg = pkg._lib.NslamLossCfg(pkg._lib.LOSS_TRACKER, 1, 1, 0.5)
    monkeypatch.setenv("NSLAM_MEDIAN_LAUNCH", "yes")
    assert L.nslam_render_loss(ctypes.byref(cfg), 4096, 4096, 4, 48, 4096, 4096, None, 4096, 4096, 4096, 4096,
                               4096, 4096, 5 * 8, None) == -1


def test_v21_gather_frame_needs_a_pose_or_a_camera(pkg):
    """A frame with neither c2w nor cam (ABI v21) is rejected before any launch."""
    L = pkg._lib.lib()
    fr = (pkg._lib.NslamFrame * 1)()
    fr[0].depth, fr[0].color = 4096, 4096
    args = [fr, 1, 10, 4096, 96, 128, 0, 96, 0, 128, 500.0, 500.0, 64.0, 48.0, None, None, 4096, 4096, 4096, 4096,
            None, None, None, None]
    assert L.nslam_gather_rays(*args) == -1
