import importlib
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) — run via gpurun")


def load_pkg():
    """The product package lives in the directory ``nice-slam_amd`` (not a valid identifier)."""
    return importlib.import_module("nice-slam_amd")


@pytest.fixture(scope="session")
def pkg():
    return load_pkg()


@pytest.fixture(scope="session")
def tiny():
    with np.load(os.path.join(GOLDEN, "tiny_scene.npz")) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def loop():
    """tests/golden/loop_fixtures.npz: loop-level vectors from the reference's own Tracker / Mapper
    code (tests/golden/make_golden_loop.py)."""
    with np.load(os.path.join(GOLDEN, "loop_fixtures.npz")) as z:
        return {k: z[k] for k in z.files}


class FixedPixels:
    """Replaces common.select_uv (src/common.py:92-107): pre-drawn flat pixel indices from a seeded
    CPU generator, in call order — the draws tests/golden/make_golden_loop.py's FixedDraws made."""

    def __init__(self, seed=11):
        import torch
        self.g = torch.Generator().manual_seed(seed)
        self.log = []

    def draw(self, n_total, n):
        import torch
        idx = torch.randint(n_total, (n,), generator=self.g)
        self.log.append(idx)
        return idx

    def __call__(self, i, j, n, depth, color, device="cuda:0", generator=None):
        i, j = i.reshape(-1), j.reshape(-1)
        idx = self.draw(i.shape[0], n).to(i.device)
        return i[idx], j[idx], depth.reshape(-1)[idx], color.reshape(-1, 3)[idx]


@pytest.fixture(scope="session")
def room0():
    with np.load(os.path.join(GOLDEN, "room0_color.npz")) as z:
        return {k: z[k] for k in z.files}


def sd_from(tiny):
    import torch
    return {k[3:]: torch.from_numpy(v) for k, v in tiny.items() if k.startswith("sd.")}


def grids_from(tiny):
    import torch
    return {k: torch.from_numpy(tiny[k]) for k in ("grid_coarse", "grid_middle", "grid_fine", "grid_color")}


def _np(x):
    if hasattr(x, "detach"):  # torch tensor (any device)
        x = x.detach().to("cpu", dtype=__import__("torch").float64).numpy()
    return np.asarray(x, dtype=np.float64).ravel()


def rel_l2(a, b):
    a, b = _np(a), _np(b)
    den = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / (den if den > 0 else 1.0))
