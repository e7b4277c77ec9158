"""ctypes binding of libnslam.so (include/nslam.h).

The product path calls the HIP kernels only through this module.  There is no CPU fallback:
if the shared library is missing, or a tensor is not on a HIP device, the call raises.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NSLAM_LIB") or os.path.join(_HERE, "libnslam.so")  # NSLAM_LIB: instrumented builds

NSLAM_OK = 0
ABI_VERSION = 23
STAGES = {"coarse": 0, "middle": 1, "fine": 2, "color": 3}
DEC_COARSE, DEC_MIDDLE, DEC_FINE, DEC_COLOR = 0, 1, 2, 3

c_float_p = ctypes.POINTER(ctypes.c_float)


class NslamGrid(ctypes.Structure):
    _fields_ = [
        ("data", ctypes.c_void_p),
        ("grad", ctypes.c_void_p),
        ("dims", ctypes.c_int32 * 3),
        ("pad_", ctypes.c_int32),
        ("lo", ctypes.c_double * 3),
        ("hi", ctypes.c_double * 3),
        ("slot", ctypes.c_void_p),  # ABI v6: frustum-compacted gradient (NULL = dense)
    ]


class NslamDecGrad(ctypes.Structure):
    _fields_ = [
        ("base", ctypes.c_void_p),
        ("w", ctypes.c_int64 * 5),
        ("b", ctypes.c_int64 * 5),
        ("wc", ctypes.c_int64 * 5),
        ("bc", ctypes.c_int64 * 5),
        ("wo", ctypes.c_int64),
        ("bo", ctypes.c_int64),
        ("B", ctypes.c_int64),
        ("count", ctypes.c_int64),
    ]


class NslamQueryCfg(ctypes.Structure):
    _fields_ = [
        ("stage", ctypes.c_int32),
        ("need_pts_grad", ctypes.c_int32),
        ("bound_lo", ctypes.c_double * 3),
        ("bound_hi", ctypes.c_double * 3),
        ("grid", NslamGrid * 4),
        ("packed", ctypes.c_void_p * 4),
        ("dgrad", NslamDecGrad * 4),
        ("rays_o", ctypes.c_void_p),
        ("rays_d", ctypes.c_void_p),
        ("z_vals", ctypes.c_void_p),
        ("n_samples", ctypes.c_int64),
        ("saved_masks", ctypes.c_void_p),
        ("defer_occ", ctypes.c_int32),  # ABI v7
        ("fwd_variant", ctypes.c_int32),  # ABI v18 (NSLAM_FWD_*)
        ("act_tape", ctypes.c_void_p),  # ABI v9: colour-decoder activation tape (NULL = none)
        ("g_h4", ctypes.c_void_p),  # ABI v17: colour decoder's d/dh4 [M][32] (NULL = none)
    ]


MAX_FRAMES = 32
ADAM_MAX_SEGS = 16
LOSS_MAPPER, LOSS_TRACKER = 0, 1


class NslamFrame(ctypes.Structure):
    _fields_ = [("depth", ctypes.c_void_p), ("color", ctypes.c_void_p), ("c2w", ctypes.c_void_p),
                ("cam", ctypes.c_void_p), ("c2w_out", ctypes.c_void_p)]


class NslamLossCfg(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int32), ("use_color", ctypes.c_int32), ("handle_dynamic", ctypes.c_int32),
                ("w_color", ctypes.c_float), ("occ_add", ctypes.c_void_p)]


class NslamDraw(ctypes.Structure):  # ABI v7 in-kernel pixel draws
    _fields_ = [("seed", ctypes.c_uint64), ("counter", ctypes.c_void_p), ("ticket", ctypes.c_void_p),
                ("world", ctypes.c_int32), ("rank", ctypes.c_int32), ("gt_max", ctypes.c_void_p),
                ("gt_max_key", ctypes.c_void_p)]


class NslamCamTail(ctypes.Structure):
    """nslam_cam_tail (ABI v23): the camera's Adam step, the iteration's loss and the best pose."""
    _fields_ = [("cam", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p), ("exp_avg_sq", ctypes.c_void_p),
                ("step", ctypes.c_void_p), ("lr", ctypes.c_float), ("beta1", ctypes.c_float),
                ("beta2", ctypes.c_float), ("eps", ctypes.c_float), ("ray_loss", ctypes.c_void_p),
                ("n_rays", ctypes.c_int64), ("loss_out", ctypes.c_void_p), ("best_loss", ctypes.c_void_p),
                ("best", ctypes.c_void_p)]


class NslamAdamSeg(ctypes.Structure):
    _fields_ = [
        ("param", ctypes.c_void_p),
        ("grad", ctypes.c_void_p),
        ("exp_avg", ctypes.c_void_p),
        ("exp_avg_sq", ctypes.c_void_p),
        ("step", ctypes.c_void_p),
        ("rows", ctypes.c_void_p),
        ("n", ctypes.c_int64),
        ("row_len", ctypes.c_int32),
        ("lr", ctypes.c_float),
        ("grad_rows", ctypes.c_int32),  # ABI v6: compact [n][row_len] gradient of a row-masked segment
        ("pad_", ctypes.c_int32),
        ("mirror_idx", ctypes.c_void_p),  # ABI v7: packed-copy slots [n][2] of a dense segment
        ("mirror", ctypes.c_void_p),
        ("n_live", ctypes.c_void_p),  # ABI v19: device int64 live count (NULL = n)
    ]


# every symbol include/nslam.h declares (tests check that the library exports all of them)
EXPORTS = (
    "nslam_pack_layout", "nslam_sample_rays", "nslam_query_fwd", "nslam_query_bwd", "nslam_query_bwd_workspace_size",
    "nslam_query_saved_size", "nslam_query_bwd_decoder", "nslam_query_bwd_decoder_workspace_size",
    "nslam_query_bwd_decoders",
    "nslam_composite_fwd", "nslam_composite_bwd", "nslam_grid_sample_fwd", "nslam_grid_sample_bwd",
    "nslam_workspace_size", "nslam_strerror", "nslam_abi_version", "nslam_gather_rays", "nslam_render_loss",
    "nslam_render_loss_workspace_size", "nslam_adam_step", "nslam_rows_pack", "nslam_rows_unpack",
    "nslam_query_fwd_ws", "nslam_query_fwd_workspace_size", "nslam_cam_grad", "nslam_cam_pose",
    "nslam_query_tape_size", "nslam_color_wgrad", "nslam_cam_grad_parts", "nslam_cam_grad_batch",
    "nslam_cam_pose_batch", "nslam_frustum_rows", "nslam_frustum_rows_workspace_size", "nslam_track_best",
    "nslam_loss_sum_best", "nslam_cam_vector_batch", "nslam_cam_grad_step",
)

_lib = None


def lib():
    """Load libnslam.so once (fails loudly when it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
                               "(make -C nice-slam_amd/csrc); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        # a stale build (older ABI, or one that lacks an export) gets the rebuild message, not an
        # AttributeError from the first missing symbol
        missing = [n for n in EXPORTS if not hasattr(L, n)]
        if missing:
            raise RuntimeError(f"{LIB_PATH} does not export {', '.join(missing)}: rebuild it "
                               "(make -C nice-slam_amd/csrc)")
        vp, i32, i64, sz = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t
        dp = ctypes.POINTER(ctypes.c_double)
        L.nslam_pack_layout.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int32), ctypes.c_int]
        L.nslam_sample_rays.argtypes = [vp, vp, vp, vp, i64, dp, dp, vp, i32, vp, i32, i32, vp, vp, sz, vp]
        L.nslam_query_fwd.argtypes = [ctypes.POINTER(NslamQueryCfg), vp, i64, vp, vp]
        L.nslam_query_fwd_ws.argtypes = [ctypes.POINTER(NslamQueryCfg), vp, i64, vp, vp, sz, vp]
        L.nslam_query_fwd_workspace_size.argtypes = [ctypes.POINTER(NslamQueryCfg), i64]
        L.nslam_query_fwd_workspace_size.restype = sz
        L.nslam_query_bwd.argtypes = [ctypes.POINTER(NslamQueryCfg), vp, i64, vp, vp, vp, sz, vp]
        L.nslam_query_bwd_workspace_size.argtypes = [ctypes.POINTER(NslamQueryCfg), i64]
        L.nslam_query_bwd_workspace_size.restype = sz
        L.nslam_query_bwd_decoder.argtypes = [ctypes.POINTER(NslamQueryCfg), i32, i32, vp, i64, vp, vp, vp, sz, vp]
        L.nslam_query_bwd_decoders.argtypes = [ctypes.POINTER(NslamQueryCfg), i32, vp, i64, vp, ctypes.POINTER(vp), vp]
        L.nslam_color_wgrad.argtypes = [ctypes.POINTER(NslamQueryCfg), vp, i64, vp, vp, sz, vp]
        L.nslam_query_bwd_decoder_workspace_size.argtypes = [ctypes.POINTER(NslamQueryCfg), i32, i64]
        L.nslam_query_bwd_decoder_workspace_size.restype = sz
        L.nslam_query_saved_size.argtypes = [i64]
        L.nslam_query_saved_size.restype = sz
        L.nslam_query_tape_size.argtypes = [i64]
        L.nslam_query_tape_size.restype = sz
        L.nslam_composite_fwd.argtypes = [vp, vp, i64, i32, vp, vp, vp, vp]
        L.nslam_composite_bwd.argtypes = [vp, vp, i64, i32, vp, vp, vp, vp, vp]
        L.nslam_grid_sample_fwd.argtypes = [vp, ctypes.POINTER(ctypes.c_int32), vp, i64, vp, vp]
        L.nslam_grid_sample_bwd.argtypes = [vp, ctypes.POINTER(ctypes.c_int32), vp, i64, vp, vp, vp, vp]
        L.nslam_workspace_size.argtypes = [ctypes.c_int, i64]
        L.nslam_workspace_size.restype = sz
        L.nslam_strerror.argtypes = [ctypes.c_int]
        L.nslam_strerror.restype = ctypes.c_char_p
        L.nslam_abi_version.restype = ctypes.c_int
        f32 = ctypes.c_float
        L.nslam_gather_rays.argtypes = [ctypes.POINTER(NslamFrame), i32, i64, vp, i32, i32, i32, i32, i32, i32,
                                        f32, f32, f32, f32, dp, dp, vp, vp, vp, vp, vp, ctypes.POINTER(NslamDraw), vp, vp]
        L.nslam_render_loss.argtypes = [ctypes.POINTER(NslamLossCfg), vp, vp, i64, i32, vp, vp, vp, vp, vp, vp, vp,
                                        vp, vp, sz, vp]
        L.nslam_render_loss_workspace_size.argtypes = [ctypes.POINTER(NslamLossCfg), i64]
        L.nslam_render_loss_workspace_size.restype = sz
        L.nslam_adam_step.argtypes = [ctypes.POINTER(NslamAdamSeg), i32, f32, f32, f32, i32, vp, vp]
        L.nslam_rows_pack.argtypes = [vp, vp, i64, i32, vp, i64, vp, vp]
        L.nslam_rows_unpack.argtypes = [vp, vp, i64, i32, vp, vp, i64, vp]
        L.nslam_cam_grad.argtypes = [vp, vp, vp, vp, vp, i64, i32, vp, vp]
        L.nslam_cam_grad_parts.argtypes = [vp, vp, ctypes.POINTER(vp), i32, vp, vp, i64, i32, vp, vp, vp, vp]
        L.nslam_cam_pose.argtypes = [vp, vp, vp]
        L.nslam_cam_grad_batch.argtypes = [vp, vp, i64, i32, ctypes.POINTER(i64), i64, ctypes.POINTER(vp), i32, vp, vp,
                                           i64, i32, vp, vp, vp, vp]
        L.nslam_cam_pose_batch.argtypes = [vp, vp, i64, i32, vp]
        L.nslam_frustum_rows.argtypes = [vp, vp, vp, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, sz, vp]
        L.nslam_frustum_rows_workspace_size.argtypes = [i64]
        L.nslam_frustum_rows_workspace_size.restype = sz
        L.nslam_track_best.argtypes = [vp, vp, vp, vp, i32, vp]
        L.nslam_loss_sum_best.argtypes = [vp, i64, vp, vp, vp, vp, i32, vp]
        L.nslam_cam_vector_batch.argtypes = [vp, i64, i32, vp, vp, vp]
        L.nslam_cam_grad_step.argtypes = [ctypes.POINTER(NslamCamTail), vp, ctypes.POINTER(vp), i32, vp, vp, i64, i32,
                                          vp, vp, vp, vp]
        if L.nslam_abi_version() != ABI_VERSION:
            raise RuntimeError(f"libnslam.so ABI {L.nslam_abi_version()} != {ABI_VERSION}: rebuild it")
        _lib = L
    return _lib


def check(rc: int, what: str):
    if rc != NSLAM_OK:
        msg = lib().nslam_strerror(rc).decode()
        raise RuntimeError(f"{what} failed: rc={rc} ({msg})")


def ptr(t):
    """Device pointer of a tensor (None → NULL); refuses host tensors (no CPU fallback)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("nice-slam_amd kernels run on the HIP device only; got a CPU tensor")
    return t.data_ptr()


def stream_ptr(device=None):
    return torch.cuda.current_stream(device).cuda_stream


def pack_layout(kind: int, nc: int = 1):
    out = (ctypes.c_int32 * 4)()
    n = lib().nslam_pack_layout(kind, nc, out, 4)
    if n != 4:
        raise RuntimeError(f"nslam_pack_layout({kind},{nc}) failed: {n}")
    return {"total": out[0], "vec": out[1], "nf": out[2], "nb": out[3]}
