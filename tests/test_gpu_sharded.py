"""Multi-rank test of the PRODUCT's ray-sharded mapping path on the device.

Two gloo ranks (processes made by mp.spawn: fresh interpreters, no exec of a GPU process) share
the one GPU of the box.  Each runs 3 colour-stage MappingEngine iterations with in-kernel pixel
draws sliced from a global batch (PixelDraws world=2: same seed, rank r gathers its slots and the
global batch's max(gt_depth) — Renderer.py:107-111,144), frustum-compacted gradients and the
SparseGradExchange all-reduce before a replicated Adam — or (ABI v16 round) the ShardedAdamExchange:
reduce-scatter, Adam on the rank's own slices of the frustum rows / colour decoder, all-gather of the
updated values, per backward branch.  Checks:
  * both ranks end with bit-identical maps (grids and colour decoder): replicated Adam on the
    same summed gradients, or every rank's slices all-gathered;
  * those maps equal a world = 1 run of the same engine on the whole global batch (float-atomic
    summation order aside) — Mapper.py:503-504 on the full batch.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, REPO

pytestmark = pytest.mark.gpu
N_PER, ITERS, SEED = 150, 3, 11


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, rank, group=None, mode="allreduce", force=False, graph=False):
    """The mapping loop of one rank on cuda:0; returns CPU copies of the final map.
    force: world 1 with the exchange's collectives issued anyway (a one-rank RCCL group);
    graph: iteration 1 eager, then one iteration captured in a hipGraph and replayed ITERS - 1 times."""
    import importlib
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    sys.path.insert(0, GOLDEN)
    P = importlib.import_module("nice-slam_amd")
    import scenes
    dev = torch.device("cuda:0")
    with np.load(os.path.join(GOLDEN, "tiny_scene.npz")) as z:
        t = {k: z[k] for k in z.files}
    bound = torch.from_numpy(t["bound"])
    sd = {k[3:]: torch.from_numpy(v) for k, v in t.items() if k.startswith("sd.") and not k.startswith("sd.coarse")}
    nice = P.NICE(c_dim=32, coarse=False, middle_grid_len=0.64, fine_grid_len=0.32, color_grid_len=0.32)
    nice.load_state_dict(sd)
    nice.set_bound(bound)
    nice = nice.to(dev)
    c = {k: torch.from_numpy(t[k]).to(dev).contiguous(memory_format=torch.channels_last_3d)
         for k in ("grid_middle", "grid_fine", "grid_color")}
    cam = scenes.TINY_CAM
    b, poses, cur = scenes.tiny_window(3)
    frames = [(torch.from_numpy(scenes.box_depth(p, cam, b, seed=500 + k)).to(dev),
               torch.from_numpy(scenes.color_image(cam, seed=600 + k)).to(dev), torch.from_numpy(p).to(dev))
              for k, p in enumerate(poses)]
    rows = {}
    for k, v in c.items():
        m = P.mapper.frustum_mask(frames[-1][2], k, v.shape[2:], frames[-1][0], bound, cam["H"], cam["W"], cam["fx"],
                                  cam["fy"], cam["cx"], cam["cy"])
        rows[k] = P.engine.frustum_rows(m)
    eng = P.engine.MappingEngine(nice, c, bound, 32, 16, device=dev, rows=rows)
    opt = P.ops.FusedAdam([{"params": [eng.decs["color"].param], "lr": 0.005}] +
                          [{"params": [c[k]], "lr": 0.005, "rows": rows[k]} for k in c])
    dec0 = eng.decs["color"].param.detach().cpu().clone()
    if world == 1 and not force:
        ex = None
    elif mode == "sharded":
        ex = P.distributed.ShardedAdamExchange(eng, opt, group=group, force_collectives=force)
    else:
        ex = P.distributed.SparseGradExchange(eng, rows, group=group, force_collectives=force)
    losses = []

    def step():
        rl, _ = eng.iteration("color", frames, None, N_PER * (2 // world), (cam["H"], cam["W"]),
                              (cam["fx"], cam["fy"], cam["cx"], cam["cy"]), opt, seed=SEED, world=world, rank=rank,
                              exchange=ex)
        return rl

    if graph:
        losses.append(float(step().sum()))
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        # thread_local: the RCCL watchdog thread's event polls must not invalidate the capture
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            rl = step()
        for _ in range(ITERS - 1):
            g.replay()
            losses.append(float(rl.sum()))
    else:
        for _ in range(ITERS):
            losses.append(float(step().sum()))
    torch.cuda.synchronize()
    out = {k: v.detach().cpu().clone() for k, v in c.items()}
    out["color_decoder"] = eng.decs["color"].param.detach().cpu().clone() - dec0
    out["losses"] = torch.tensor(losses, dtype=torch.float64)
    return out


def _worker(rank, world, port, path, mode):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = _run(world, rank, mode=mode)
        torch.save(res, os.path.join(path, f"rank{rank}.pt"))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["allreduce", "sharded"])
def test_two_rank_sharded_engine_matches_single_rank(tmp_path, mode):
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path), mode), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    for k in r0:
        if k != "losses":
            assert torch.equal(r0[k], r1[k]), k   # identical summed gradients / all-gathered updates
    full = _run(1, 0)
    with np.load(os.path.join(GOLDEN, "tiny_scene.npz")) as z:
        start = {k: torch.from_numpy(z[k]) for k in ("grid_middle", "grid_fine", "grid_color")}
    # per-rank losses are shard sums: together they are the full batch's loss
    np.testing.assert_allclose((r0["losses"] + r1["losses"]).numpy(), full["losses"].numpy(), rtol=1e-5)
    for k, s in start.items():
        d_sh, d_full = r0[k] - s, full[k] - s
        assert float(d_full.abs().max()) > 0, k
        rel = float((d_sh - d_full).norm() / d_full.norm())
        assert rel < 1e-3, (k, rel)
    rel = float((r0["color_decoder"] - full["color_decoder"]).norm() / full["color_decoder"].norm())
    assert float(full["color_decoder"].abs().max()) > 0 and rel < 1e-3, rel


def _rccl1_worker(rank, port, path, mode):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        res = _run(1, 0, mode=mode, force=True, graph=True)
        res["backend"] = torch.tensor([dist.get_backend() == "nccl"])
        torch.save(res, os.path.join(path, "rccl1.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["allreduce", "sharded"])
def test_world1_rccl_exchange_in_hipgraph_is_identity(tmp_path, mode):
    """The N > 1 exchange path on one GPU: a one-rank RCCL group, the exchange's collectives issued
    anyway (force_collectives: all-reduce, or reduce-scatter + sharded Adam + all-gather per backward
    branch on two communicators) and captured with the iteration in a hipGraph.  At world 1 every
    collective is an identity, so the map after 3 iterations equals the no-exchange run's — up to
    float-atomic summation order in the grid-gradient scatter (rel 1e-5 of the map's change)."""
    port = _free_port()
    mp.spawn(_rccl1_worker, args=(port, str(tmp_path), mode), nprocs=1, join=True)
    r = torch.load(tmp_path / "rccl1.pt", weights_only=True)
    assert bool(r.pop("backend"))
    ref = _run(1, 0, graph=True)
    with np.load(os.path.join(GOLDEN, "tiny_scene.npz")) as z:
        start = {k: torch.from_numpy(z[k]) for k in ("grid_middle", "grid_fine", "grid_color")}
    np.testing.assert_allclose(r["losses"].numpy(), ref["losses"].numpy(), rtol=1e-6)
    for k, s0 in start.items():
        d, d_ref = r[k] - s0, ref[k] - s0
        assert float(d_ref.abs().max()) > 0, k
        assert float((d - d_ref).norm() / d_ref.norm()) <= 1e-5, k
    rel = float((r["color_decoder"] - ref["color_decoder"]).norm() / ref["color_decoder"].norm())
    assert rel <= 1e-5, rel
