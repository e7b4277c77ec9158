"""CPU-side checks of the boundary: libnslam.so loads, exports every symbol include/nslam.h
declares, and the Python pack layout agrees with the C++ one (no GPU calls)."""
import ctypes
import os
import re

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
    assert L.nslam_abi_version() == 3
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


def test_no_cpu_fallback(pkg):
    import torch
    with pytest.raises(RuntimeError, match="HIP device"):
        pkg.ops.composite(torch.zeros(2, 4, 4), torch.zeros(2, 4, dtype=torch.float64))
