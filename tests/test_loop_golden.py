"""CPU checks against the loop-level golden vectors (tests/golden/loop_fixtures.npz, made by
running the reference's own Tracker / Mapper / common code, tests/golden/make_golden_loop.py):

  * the oracle's camera, tracker-loss and mapper-loss restatements (a3, a13, a14) are pinned;
  * the product's host-side torch logic — frustum voxel selection and keyframe-overlap scores
    (Mapper.py:93-228, §8 a17 / f3) — equals the reference on CPU (the GPU tests repeat it on
    the device).
"""
import importlib
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN, FixedPixels, rel_l2
from oracle import nslam_oracle as orc

sys.path.insert(0, GOLDEN)
import scenes  # noqa: E402


def test_camera_from_tensor_pinned(loop):
    cams = torch.from_numpy(loop["camera.cam"])
    ref = torch.from_numpy(loop["camera.c2w"])
    got = torch.stack([orc.camera_from_tensor(c) for c in cams])
    assert torch.equal(got, ref)


def test_camera_chain_vjp_pinned(loop):
    """d loss / d 7-vector through get_camera_from_tensor → get_rays_from_uv → pts = o + d·z."""
    cam = dict(scenes.ROOM0_CAM)
    for b in range(loop["camera.cam"].shape[0]):
        t = torch.from_numpy(loop["camera.cam"][b]).clone().requires_grad_(True)
        c2w = orc.camera_from_tensor(t)
        ro, rd = orc.rays_from_uv(torch.from_numpy(loop["camera.i"][b]), torch.from_numpy(loop["camera.j"][b]), c2w,
                                  cam["fx"], cam["fy"], cam["cx"], cam["cy"])
        assert torch.equal(rd.detach(), torch.from_numpy(loop["camera.rays_d"][b]))
        z = torch.from_numpy(loop["camera.z"][b])
        pts = ro[:, None, :] + rd[:, None, :] * z[..., None]
        (g,) = torch.autograd.grad(pts, (t,), torch.from_numpy(loop["camera.g_pts"][b]))
        assert rel_l2(g, loop["camera.grad_cam"][b]) < 1e-6, b


@pytest.mark.parametrize("case,hd", [("tloss_hd", True), ("tloss_nohd", False)])
def test_tracker_loss_pinned(loop, case, hd):
    raw = torch.from_numpy(loop[case + ".raw"]).clone().requires_grad_(True)
    z = torch.from_numpy(loop[case + ".z"])
    depth, var, color, _ = orc.composite(raw, z)
    loss = orc.tracker_loss(depth, var, color, torch.from_numpy(loop[case + ".gt_depth"]),
                            torch.from_numpy(loop[case + ".gt_color"]), handle_dynamic=hd)
    loss.backward()
    assert abs(float(loss) - float(loop[case + ".loss"])) <= 1e-9 * abs(float(loop[case + ".loss"]))
    assert rel_l2(raw.grad, loop[case + ".g_raw"]) < 1e-6


@pytest.mark.parametrize("stage", ["color", "middle"])
def test_mapper_loss_pinned(loop, stage):
    case = "mloss_" + stage
    raw = torch.from_numpy(loop[case + ".raw"]).clone().requires_grad_(True)
    z = torch.from_numpy(loop[case + ".z"])
    depth, _, color, _ = orc.composite(raw, z)
    loss = orc.mapper_loss(depth, color, torch.from_numpy(loop[case + ".gt_depth"]),
                           torch.from_numpy(loop[case + ".gt_color"]), stage)
    loss.backward()
    assert abs(float(loss) - float(loop[case + ".loss"])) <= 1e-9 * abs(float(loop[case + ".loss"]))
    assert rel_l2(raw.grad, loop[case + ".g_raw"]) < 1e-6


@pytest.fixture(scope="module")
def P():
    return importlib.import_module("nice-slam_amd")


def test_frustum_mask_host_matches_reference(loop, P):
    """mapper.frustum_mask (torch, here on CPU) == Mapper.get_mask_from_c2w at room0 grid shapes."""
    b, _, cur = scenes.room0_window()
    cam = scenes.ROOM0_CAM
    depth = torch.from_numpy(scenes.box_depth(cur, cam, b, seed=int(loop["frustum.depth_seed"])))
    for key in ("grid_middle", "grid_fine", "grid_color"):
        shp = tuple(int(v) for v in loop["frustum.shape." + key])
        m = P.mapper.frustum_mask(torch.from_numpy(cur), key, shp, depth, torch.from_numpy(b), cam["H"], cam["W"],
                                  cam["fx"], cam["fy"], cam["cx"], cam["cy"])
        ref = loop["frustum.mask." + key]
        assert ref.sum() > 0 and (~ref).sum() > 0
        np.testing.assert_array_equal(m.numpy(), ref, err_msg=key)


def overlap_mapper(P, device):
    """A drop-in Mapper with only what keyframe selection reads (room0 camera)."""
    mp = object.__new__(P.Mapper)
    cam = scenes.ROOM0_CAM
    mp.H, mp.W, mp.fx, mp.fy, mp.cx, mp.cy = cam["H"], cam["W"], cam["fx"], cam["fy"], cam["cx"], cam["cy"]
    mp.device, mp.generator = device, None
    return mp


def test_keyframe_overlap_host_matches_reference(loop, P, monkeypatch):
    b, poses, cur = scenes.room0_window()
    cam = scenes.ROOM0_CAM
    depth = torch.from_numpy(scenes.box_depth(cur, cam, b, seed=int(loop["overlap.depth_seed"])))
    color = torch.from_numpy(scenes.color_image(cam, seed=int(loop["overlap.color_seed"])))
    kf = [{"est_c2w": torch.from_numpy(p)} for p in poses]
    mp = overlap_mapper(P, "cpu")
    monkeypatch.setattr(P.common, "select_uv", FixedPixels(int(loop["overlap.draw_seed"])))
    scores = mp.keyframe_overlap_scores(color, depth, torch.from_numpy(cur), kf)
    np.testing.assert_array_equal(np.asarray(scores), loop["overlap.scores"])
    monkeypatch.setattr(P.common, "select_uv", FixedPixels(int(loop["overlap.draw_seed"])))
    np.random.seed(int(loop["overlap.np_seed"]))
    sel = mp.keyframe_selection_overlap(color, depth, torch.from_numpy(cur), kf, int(loop["overlap.k"]))
    assert [int(s) for s in sel] == [int(s) for s in loop["overlap.selected"]]


def test_scene_helpers_deterministic():
    """The shared frame generator is pure numpy: the same seed gives the same bits."""
    b, poses, cur = scenes.room0_window()
    a = scenes.box_depth(cur, scenes.ROOM0_CAM, b, seed=5)
    c = scenes.box_depth(cur, scenes.ROOM0_CAM, b, seed=5)
    assert np.array_equal(a, c) and a.dtype == np.float32 and (a == 0).any() and (a > 0).mean() > 0.9
    assert os.path.exists(os.path.join(GOLDEN, "make_golden_loop.py"))
