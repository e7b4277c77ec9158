"""nice-slam_amd — NICE-SLAM's volumetric-rendering hot path on MI355X (gfx950).

Host code mirrors the reference's API (src/common.py, src/conv_onet/models/decoder.py,
src/utils/Renderer.py, Tracker.optimize_cam_in_batch, Mapper.optimize_map); the compute runs in
hand-written HIP kernels in libnslam.so (csrc/), bound through the C-ABI of include/nslam.h.
The directory name is not a Python identifier: import with importlib.import_module("nice-slam_amd").
"""
import sys as _sys

from . import _lib, common, datasets, decoder, distributed, engine, mapper, ops, packing, renderer, slam, tracker  # noqa: F401,E501
from .datasets import get_dataset  # noqa: F401
from .decoder import NICE, MLP, MLP_no_xyz  # noqa: F401
from .mapper import Mapper  # noqa: F401
from .renderer import Renderer  # noqa: F401
from .tracker import Tracker  # noqa: F401

_sys.modules.setdefault("nice_slam_amd", _sys.modules[__name__])

__all__ = ["NICE", "MLP", "MLP_no_xyz", "Renderer", "Tracker", "Mapper", "get_dataset", "common", "datasets", "decoder",
           "distributed", "mapper", "ops", "packing", "renderer", "slam", "tracker"]
