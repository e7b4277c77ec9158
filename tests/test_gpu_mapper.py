"""Mapper.optimize_map on the fused engine: the hipGraph path against the eager path, and the fused
path against the autograd drop-in (src/Mapper.py:230-540).

  * graphs vs eager: the same device pixel draws (the draw stream is rewound after the capture
    warm-ups), BA over a 3-frame window with frustum selection, two calls — the second replays the
    graphs the first captured, with another frustum selection bound on the device.  Same kernels in
    the same order; only the float-atomic grid scatter orders sums differently, which Adam's
    normalisation turns into relative update differences of ~1e-5.
  * fused vs autograd: both through the product's select_uv (pinned draws), the coarse mapper
    (Mapper.py:403-404, 482-484: stage 'coarse', no gt in the sampler, dense coarse grid).
Tolerances: losses rtol 1e-4 (graphs) / 2e-3 (fused vs autograd, tests/test_gpu_dropins.py), parameter
updates rel-L2 1e-3.
"""
import importlib

import numpy as np
import pytest
import torch

from conftest import FixedPixels, rel_l2
from test_gpu_dropins import Scene, _nudged, base_cfg

pytestmark = pytest.mark.gpu
P = importlib.import_module("nice-slam_amd")


def _run_two_calls(tiny, monkeypatch, graphs, ba=True):
    sc = Scene(tiny)
    cfg = base_cfg()
    cfg["mapping"].update(frustum_feature_selection=True, pixels=600)
    slam = sc.slam(cfg)
    mp = P.Mapper(cfg, None, slam)
    mp.BA = ba
    mp.graphs = graphs
    mp._draw_seed = 1234
    mp.loss_history = []
    monkeypatch.setattr(mp, "keyframe_selection_overlap", lambda *a, **k: [0])
    est = [sc.c2w.clone(), _nudged(sc.c2w, 0.01, (0.01, -0.005, 0.0))]
    kf = [{"gt_c2w": sc.c2w, "idx": i, "color": sc.color, "depth": sc.depth, "est_c2w": est[i].clone()}
          for i in range(2)]
    outs, ngraphs = [], []
    for call, (ang, t) in enumerate(((-0.008, (0.0, 0.006, 0.004)), (0.012, (0.004, -0.002, 0.003)))):
        cur = _nudged(sc.c2w, ang, t)
        out = mp.optimize_map(6, 1.0, 2 + call, sc.color, sc.depth, sc.c2w, kf, [0, 1], cur.clone())
        outs.append(out.detach().cpu() if out is not None else torch.zeros(4, 4))
        ngraphs.append(sum(1 for k in mp._graphs if k[0] == "stage"))
    torch.cuda.synchronize()
    grids = {k: v.detach().cpu().clone() for k, v in slam.shared_c.items()}
    dec = torch.cat([p.detach().reshape(-1).cpu() for p in mp.decoders.color_decoder.parameters()])
    return {"losses": [float(x) for x in mp.loss_history], "grids": grids, "dec": dec, "outs": outs,
            "kf1": kf[1]["est_c2w"].detach().cpu(), "ngraphs": ngraphs, "g0": {k: v.cpu() for k, v in sc.grids.items()}}


@pytest.mark.parametrize("ba", [True, False])
def test_optimize_map_graphs_match_eager(tiny, monkeypatch, ba):
    """(ba=False: the captured runs also hold the ray prefetch chain of each stage run.)"""
    eager = _run_two_calls(tiny, monkeypatch, graphs=False, ba=ba)
    graph = _run_two_calls(tiny, monkeypatch, graphs=True, ba=ba)
    assert eager["ngraphs"] == [0, 0]
    # the first call captured one graph per stage run (middle, fine, colour); the second replayed them
    assert graph["ngraphs"][0] == 3 and graph["ngraphs"][1] == 3
    assert len(graph["losses"]) == len(eager["losses"]) == 12
    np.testing.assert_allclose(graph["losses"], eager["losses"], rtol=1e-4)
    report = {}
    for k, g in graph["grids"].items():
        report[k] = rel_l2(g - graph["g0"][k], eager["grids"][k] - eager["g0"][k])
    report["color_decoder"] = rel_l2(graph["dec"], eager["dec"])
    for i, (a, b) in enumerate(zip(graph["outs"], eager["outs"])):
        report[f"cur{i}"] = rel_l2(a, b)
    report["kf1"] = rel_l2(graph["kf1"], eager["kf1"])
    print(report)
    assert all(v < 1e-3 for v in report.values()), report


def test_coarse_mapper_fused_matches_autograd(tiny, monkeypatch):
    """The coarse mapper (coarse grid, global keyframe selection) on the fused engine vs the autograd
    drop-in, on the same pinned pixel draws."""
    res = {}
    for path in ("fused", "autograd"):
        sc = Scene(tiny)
        cfg = base_cfg()
        cfg["coarse"] = True
        cfg["mapping"]["stage"]["coarse"] = {"decoders_lr": 0.0, "coarse_lr": 0.001, "middle_lr": 0.0, "fine_lr": 0.0,
                                             "color_lr": 0.0}
        cfg["mapping"].update(frustum_feature_selection=True, pixels=400)
        nice = P.NICE(c_dim=32, coarse=True, coarse_grid_len=2.0, middle_grid_len=0.64, fine_grid_len=0.32,
                      color_grid_len=0.32)
        nice.load_state_dict({k: v.clone() for k, v in sc.sd.items()})
        nice.set_bound(sc.bound)
        slam = sc.slam(cfg)
        slam.shared_decoders = nice.to(sc.dev)
        slam.shared_c["grid_coarse"] = torch.from_numpy(tiny["grid_coarse"]).to(sc.dev).contiguous(
            memory_format=torch.channels_last_3d)
        g0 = slam.shared_c["grid_coarse"].detach().cpu().clone()
        mp = P.Mapper(cfg, None, slam, coarse_mapper=True)
        mp.fused = path == "fused"
        mp.loss_history = []
        monkeypatch.setattr(P.common, "select_uv", FixedPixels(seed=21))
        kf = [{"gt_c2w": sc.c2w, "idx": 0, "color": sc.color, "depth": sc.depth, "est_c2w": sc.c2w.clone()}]
        np.random.seed(5)
        mp.optimize_map(4, 1.0, 1, sc.color, sc.depth, sc.c2w, kf, [0], sc.c2w.clone())
        torch.cuda.synchronize()
        res[path] = ([float(x) for x in mp.loss_history], slam.shared_c["grid_coarse"].detach().cpu() - g0,
                     {k: (slam.shared_c[k].detach().cpu() - sc.grids[k]).abs().max().item()
                      for k in ("grid_middle", "grid_fine", "grid_color")})
        monkeypatch.undo()
    lf, gf, other_f = res["fused"]
    la, ga, other_a = res["autograd"]
    np.testing.assert_allclose(lf, la, rtol=2e-3)
    assert float(ga.abs().max()) > 0
    assert rel_l2(gf, ga) < 1e-3, rel_l2(gf, ga)
    # only the coarse grid is optimised by the coarse mapper
    assert max(other_f.values()) == 0.0 and max(other_a.values()) == 0.0


def test_tracker_graph_matches_eager_device_draws(tiny):
    """Tracker.track_frame's captured camera loop (one hipGraph per frame, device draws) == the same loop
    run eagerly on the tracking engine with the same draw stream — bit for bit (the camera chain is
    deterministic: no float atomics), on the frame that captures the graph and on one that replays it."""
    cfg = base_cfg()
    sc = Scene(tiny)
    c2w = torch.cat([sc.c2w[:3], torch.tensor([[0, 0, 0, 1.0]])], 0).cuda()
    pres = []
    for d in (0.02, -0.015):
        pre = c2w.clone()
        pre[:3, 3] += d
        pres.append(pre)
    tr = P.Tracker(cfg, None, sc.slam(cfg))
    tr._draw_seed = 77
    got = [tr.track_frame(k + 1, sc.color.cuda(), sc.depth.cuda(), c2w, pre_c2w=pre) for k, pre in enumerate(pres)]
    assert len(tr._graphs) == 1
    # eager replica: the same engine calls, draws from the same stream (counter 0, advancing per iteration)
    tr2 = P.Tracker(cfg, None, sc.slam(cfg))
    tr2.update_para_from_mapping()
    eng = tr2.engine()
    ref = []
    for pre in pres:
        # (the graph forms the guess's 7-vector and the result pose with nslam_cam_vector_batch / nslam_cam_pose)
        cam = P.ops.cam_vector_batch(pre[None].contiguous(), torch.empty(1, 7, device="cuda"))[0]
        cam = cam.clone().requires_grad_(True)
        opt = P.ops.FusedAdam([{"params": [cam], "lr": cfg["tracking"]["lr"]}])
        best, best_loss = cam.detach().clone(), torch.full((), float("inf"), dtype=torch.float64, device="cuda")
        for _ in range(cfg["tracking"]["iters"]):
            loss = eng.iteration(cam, sc.depth.cuda(), sc.color.cuda(), None, opt, n=cfg["tracking"]["pixels"], seed=77)
            better = loss < best_loss
            best_loss = torch.where(better, loss, best_loss)
            best = torch.where(better, cam.detach(), best)
        pose = torch.eye(4, device="cuda")
        P.ops.cam_pose(best.contiguous(), pose[:3])
        ref.append(pose)
    for a, b in zip(got, ref):
        assert torch.equal(a, b), (a - b).abs().max()
    assert not torch.equal(got[0], pres[0])  # the loop moved the pose
