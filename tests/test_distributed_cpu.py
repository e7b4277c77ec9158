"""World-size-2 gloo test of the ray-sharded mapping step (CPU).

Product code under test: nice-slam_amd/distributed.py (shard_range, global_max, allreduce_grads).
The per-shard compute is the oracle (test infrastructure), injected here: the HIP path needs a GPU.
Check: sum over ranks of shard gradients == full-batch gradient, with the sampler's batch-global
max(gt_depth) taken over the full batch (all-reduced), for grids, decoder params and a loss value.
"""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _step(sd, grids, ro, rd, gt, gc, bound, gt_max):
    from oracle import nslam_oracle as orc
    d, v, c = orc.render_batch_ray(sd, grids, rd, ro, "color", bound, gt, gt_max=gt_max)
    loss = orc.mapper_loss(d, c, gt, gc, "color")
    loss.backward()
    return loss.detach()


def _worker(rank, world, port, out_path):
    import sys
    sys.path.insert(0, REPO)
    import importlib
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    D = importlib.import_module("nice-slam_amd").distributed
    with np.load(os.path.join(GOLDEN, "tiny_scene.npz")) as z:
        t = {k: z[k] for k in z.files}
    bound = torch.from_numpy(t["bound"])
    sd = {k[3:]: torch.from_numpy(v).clone().requires_grad_(k.startswith("sd.color_decoder"))
          for k, v in t.items() if k.startswith("sd.")}
    grids = {k: torch.from_numpy(t[k]).clone().contiguous(memory_format=torch.channels_last_3d).requires_grad_(True)
             for k in ("grid_middle", "grid_fine", "grid_color")}
    ro, rd, gt = (torch.from_numpy(t[k]) for k in ("rays_o", "rays_d", "gt_depth"))
    gc = torch.rand(ro.shape[0], 3, generator=torch.Generator().manual_seed(5))
    s, e = D.shard_range(ro.shape[0], rank, world)
    gmax = D.global_max(gt[s:e])
    loss = _step(sd, grids, ro[s:e], rd[s:e], gt[s:e], gc[s:e], bound, gmax)
    params = list(grids.values()) + [v for v in sd.values() if v.requires_grad]
    D.allreduce_grads(params, bucket_bytes=1 << 16)
    dist.all_reduce(loss)
    if rank == 0:
        # full batch on one rank, same code path
        sd2 = {k: v.detach().clone().requires_grad_(v.requires_grad) for k, v in sd.items()}
        g2 = {k: v.detach().clone().contiguous(memory_format=torch.channels_last_3d).requires_grad_(True)
              for k, v in grids.items()}
        loss_full = _step(sd2, g2, ro, rd, gt, gc, bound, None)
        res = {"loss": float(loss), "loss_full": float(loss_full)}
        for k in grids:
            a, b = grids[k].grad.double(), g2[k].grad.double()
            res[k] = float((a - b).norm() / b.norm())
        for k in sd:
            if sd[k].requires_grad:
                a, b = sd[k].grad.double(), sd2[k].grad.double()
                res[k] = float((a - b).norm() / max(float(b.norm()), 1e-30))
        torch.save(res, out_path)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_mapping_grads_equal_full_batch(tmp_path):
    out = str(tmp_path / "res.pt")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    res = torch.load(out)
    assert abs(res["loss"] - res["loss_full"]) <= 1e-9 * abs(res["loss_full"]) + 1e-9, res
    for k, v in res.items():
        if k.startswith("grid_") or k.startswith("color_decoder"):
            assert v < 1e-5, (k, v)


def test_shard_range_covers_everything():
    import importlib
    D = importlib.import_module("nice-slam_amd").distributed
    for n in (0, 1, 7, 64, 1001):
        for w in (1, 2, 3, 8):
            rs = [D.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(e - s for s, e in rs) - min(e - s for s, e in rs) <= 1


# ---- frustum-compacted gradient exchange (distributed.SparseGradExchange) ---------------------

def _torch_rows_pack(grid_flat, rows, tail, out):
    """CPU restatement of nslam_rows_pack (include/nslam.h) for the host-logic test."""
    n = rows.numel() if rows is not None else 0
    if n:
        out[:n * 32].copy_(grid_flat.view(-1, 32)[rows.long()].reshape(-1))
    if tail is not None:
        out[n * 32:n * 32 + tail.numel()].copy_(tail)


def _torch_rows_unpack(buf, rows, grid_flat, tail):
    n = rows.numel() if rows is not None else 0
    if n:
        grid_flat.view(-1, 32)[rows.long()] = buf[:n * 32].view(-1, 32)
    if tail is not None:
        tail.copy_(buf[n * 32:n * 32 + tail.numel()])


class _FakeEngine:
    """The engine attributes SparseGradExchange reads: grids `c`, flat `gbuf`, decoder grads."""

    def __init__(self, shapes, n_dec, rank):
        from types import SimpleNamespace
        g = torch.Generator().manual_seed(100 + rank)
        self.c = {k: torch.zeros(1, 32, *s).contiguous(memory_format=torch.channels_last_3d) for k, s in shapes.items()}
        self.gbuf = torch.randn(sum(v.numel() for v in self.c.values()), generator=g)
        self.decs = {"color": SimpleNamespace(grad=torch.randn(n_dec, generator=g))}


def _exchange_worker(rank, world, port, out_path):
    import sys
    sys.path.insert(0, REPO)
    import importlib
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    D = importlib.import_module("nice-slam_amd").distributed
    shapes = {"grid_middle": (3, 4, 5), "grid_fine": (5, 6, 7), "grid_color": (5, 6, 7)}
    rows = {"grid_middle": torch.tensor([0, 7, 59], dtype=torch.int32),
            "grid_fine": torch.tensor([1, 2, 3, 100, 209], dtype=torch.int32),
            "grid_color": torch.tensor([5, 150], dtype=torch.int32)}
    eng = _FakeEngine(shapes, 37, rank)
    before_g, before_d = eng.gbuf.clone(), eng.decs["color"].grad.clone()
    ex = D.SparseGradExchange(eng, rows, pack=_torch_rows_pack, unpack=_torch_rows_unpack)
    keys = ("grid_middle", "grid_fine", "grid_color")
    ex(keys, ("color",))
    torch.save({"before_g": before_g, "before_d": before_d, "after_g": eng.gbuf, "after_d": eng.decs["color"].grad,
                "bytes": ex.payload_bytes(keys, ("color",))}, f"{out_path}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_sparse_exchange_sums_frustum_rows_only(tmp_path):
    out = str(tmp_path / "ex")
    mp.spawn(_exchange_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r = [torch.load(f"{out}.{k}") for k in range(2)]
    off = {"grid_middle": 0, "grid_fine": 60, "grid_color": 270}   # rows of 32 floats
    sel = {"grid_middle": [0, 7, 59], "grid_fine": [1, 2, 3, 100, 209], "grid_color": [5, 150]}
    flat_rows = sorted(off[k] + i for k in sel for i in sel[k])
    assert r[0]["bytes"] == (len(flat_rows) * 32 + 37) * 4
    total_g = r[0]["before_g"].view(-1, 32) + r[1]["before_g"].view(-1, 32)
    for k in range(2):
        after = r[k]["after_g"].view(-1, 32)
        before = r[k]["before_g"].view(-1, 32)
        m = torch.zeros(after.shape[0], dtype=torch.bool)
        m[flat_rows] = True
        assert torch.equal(after[m], total_g[m])          # frustum rows: summed over ranks
        assert torch.equal(after[~m], before[~m])         # other rows: untouched
        assert torch.equal(r[k]["after_d"], r[0]["before_d"] + r[1]["before_d"])


def _compact_exchange_worker(rank, world, port, out_path, inplace=False):
    """Engine with frustum-compacted gradients (engine.rows set): the compact [n_rows, 32] grid
    gradients and the decoder gradients are summed over ranks as they are."""
    import sys
    sys.path.insert(0, REPO)
    import importlib
    from types import SimpleNamespace
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    D = importlib.import_module("nice-slam_amd").distributed
    g = torch.Generator().manual_seed(200 + rank)
    rows = {"grid_middle": torch.tensor([0, 7, 59], dtype=torch.int32),
            "grid_fine": torch.tensor([1, 2, 3, 100, 209], dtype=torch.int32)}
    gall = torch.randn(8 * 32 + 11, generator=g)
    gbuf = gall[:256]
    # inplace: the decoder gradient follows the grid rows in one buffer (MappingEngine.gall layout)
    dgrad = gall[256:] if inplace else gall[256:].clone()
    eng = SimpleNamespace(c={"grid_middle": None, "grid_fine": None}, gbuf=gbuf, rows=rows,
                          ggrad={"grid_middle": gbuf[:96].view(-1, 32), "grid_fine": gbuf[96:].view(-1, 32)},
                          decs={"color": SimpleNamespace(grad=dgrad)})
    before_g, before_d = gbuf.clone(), eng.decs["color"].grad.clone()
    ex = D.SparseGradExchange.__new__(D.SparseGradExchange)
    ex.engine, ex.group, ex.rows, ex._plan, ex.force = eng, None, {}, {}, False
    ex.pack, ex.unpack = _torch_rows_pack, _torch_rows_unpack
    if inplace:  # one contiguous span: all-reduced where it lies, no pack/unpack copies
        def _no_copy(*a):
            raise AssertionError("in-place exchange must not pack/unpack")
        ex.pack = ex.unpack = _no_copy
    keys = ("grid_middle", "grid_fine")
    ex(keys, ("color",))
    torch.save({"before_g": before_g, "before_d": before_d, "after_g": gbuf, "after_d": eng.decs["color"].grad,
                "bytes": ex.payload_bytes(keys, ("color",))}, f"{out_path}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("inplace", [False, True])
def test_compact_exchange_sums_compact_rows(tmp_path, inplace):
    out = str(tmp_path / "cx")
    mp.spawn(_compact_exchange_worker, args=(2, _free_port(), out, inplace), nprocs=2, join=True)
    r = [torch.load(f"{out}.{k}") for k in range(2)]
    assert r[0]["bytes"] == (8 * 32 + 11) * 4
    for k in range(2):
        assert torch.equal(r[k]["after_g"], r[0]["before_g"] + r[1]["before_g"])
        assert torch.equal(r[k]["after_d"], r[0]["before_d"] + r[1]["before_d"])


# ---- sharded optimiser step (distributed.ShardedAdamExchange) -------------------------------------

def _torch_adam_slices(opt, D):
    """CPU restatement of nslam_adam_step over the exchange's slices (torch.optim.Adam's element
    update, nslam_dev.h adam_one, step count per parameter advanced once per call)."""
    def run(slices, span, key):
        b1, b2 = opt.betas
        for p, rows, a0, b0, a in slices:
            ex, ex2, step = opt.state_of(p)
            t = float(step) + 1.0
            lr = float(opt.group_of(p)["lr"])
            g = span[a:a + (b0 - a0)]
            m, v = ex[a0:b0], ex2[a0:b0]
            m.mul_(b1).add_(g, alpha=1 - b1)
            v.mul_(b2).addcmul_(g, g, value=1 - b2)
            den = v.sqrt() / math.sqrt(1 - b2 ** t) + opt.eps
            upd = (lr / (1 - b1 ** t)) * (m / den)
            if rows is not None:
                D._storage(p.data).view(-1, 32)[rows[a0 // 32:b0 // 32].long()] -= upd.view(-1, 32)
            else:
                D._storage(p.data)[a0:b0] -= upd
            step += 1
    return run


def _sharded_setup(rank):
    import importlib
    import sys
    sys.path.insert(0, REPO)
    P = importlib.import_module("nice-slam_amd")
    with np.load(os.path.join(GOLDEN, "tiny_scene.npz")) as z:
        t = {k: z[k] for k in z.files}
    bound = torch.from_numpy(t["bound"])
    sd = {k[3:]: torch.from_numpy(v) for k, v in t.items() if k.startswith("sd.") and not k.startswith("sd.coarse")}
    nice = P.NICE(c_dim=32, coarse=False, middle_grid_len=0.64, fine_grid_len=0.32, color_grid_len=0.32)
    nice.load_state_dict(sd)
    nice.set_bound(bound)
    c = {k: torch.from_numpy(t[k]).contiguous(memory_format=torch.channels_last_3d)
         for k in ("grid_middle", "grid_fine", "grid_color")}
    # frustum rows: uneven counts (not multiples of the world size: the padding is exercised)
    rows = {k: torch.arange(i, v[0, 0].numel(), 3 + i, dtype=torch.int32) for i, (k, v) in enumerate(c.items())}
    eng = P.engine.MappingEngine(nice, c, bound, 32, 16, device="cpu", rows=rows)
    opt = P.ops.FusedAdam([{"params": [eng.decs["color"].param], "lr": 0.005}] +
                          [{"params": [c[k]], "lr": 0.01, "rows": rows[k]} for k in c])
    return P, eng, opt, c, rows


def _fill_grads(eng, rank, it):
    g = torch.Generator().manual_seed(1000 * it + rank)
    for k, v in eng.ggrad.items():
        v.copy_(torch.randn(v.shape, generator=g))
    d = eng.decs["color"].grad
    d.copy_(torch.randn(d.shape, generator=g))


def _sharded_worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    P, eng, opt, c, rows = _sharded_setup(rank)
    D = P.distributed
    ex = D.ShardedAdamExchange(eng, opt, pack=_torch_rows_pack, unpack=_torch_rows_unpack,
                               adam_slices=_torch_adam_slices(opt, D))
    keys = ("grid_middle", "grid_fine", "grid_color")
    zero = []
    for it in range(3):
        _fill_grads(eng, rank, it)
        ex.branch(["middle", "fine"], "grids", keys, ("color",))
        ex.branch(["color"], "all", keys, ("color",))
        zero.append(float(eng.gall.abs().sum()))  # every consumed gradient entry is zeroed
    out = {k: v.clone() for k, v in c.items()}
    out["dec"] = eng.decs["color"].param.clone()
    out["packed"] = eng.decs["color"].packed.clone()
    out["zero"] = torch.tensor(zero)
    out["pad"] = torch.tensor([eng.ggrad_pad[k].numel() // 32 for k in keys])
    torch.save(out, f"{out_path}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_adam_exchange_equals_replicated_step(tmp_path):
    """ShardedAdamExchange (reduce-scatter, Adam on this rank's slices, all-gather) over 2 gloo ranks
    == summing both ranks' gradients and stepping Adam on everything (world = 1): grids, colour
    decoder and its packed copy, for 3 iterations (step counts advance per parameter)."""
    out = str(tmp_path / "sh")
    mp.spawn(_sharded_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r = [torch.load(f"{out}.{k}") for k in range(2)]
    for k in r[0]:
        assert torch.equal(r[0][k], r[1][k]), k                  # all-gathered: identical on every rank
    assert float(r[0]["zero"].abs().max()) == 0.0
    assert all(int(n) % 2 == 0 for n in r[0]["pad"])          # whole rows per shard
    P, eng, opt, c, rows = _sharded_setup(0)
    D = P.distributed
    adam = _torch_adam_slices(opt, D)
    keys = ("grid_middle", "grid_fine", "grid_color")
    for it in range(3):
        grads = {}
        for rank in range(2):
            _fill_grads(eng, rank, it)
            for k in keys:
                grads[k] = grads.get(k, 0) + eng.ggrad[k].clone()
            grads["dec"] = grads.get("dec", 0) + eng.decs["color"].grad.clone()
        sl, span = [], []
        off = 0
        for k in keys:
            n = rows[k].numel() * 32
            sl.append((c[k], rows[k], 0, n, off))
            span.append(grads[k].reshape(-1))
            off += n
        adam(sl, torch.cat(span), None)
        p = eng.decs["color"].param
        adam([(p, None, 0, p.numel(), 0)], grads["dec"], None)
    eng.decs["color"].repack()
    for k in keys:
        assert torch.allclose(r[0][k], c[k], rtol=0, atol=1e-7), k
    assert torch.allclose(r[0]["dec"], eng.decs["color"].param, rtol=0, atol=1e-7)
    assert torch.allclose(r[0]["packed"], eng.decs["color"].packed, rtol=0, atol=1e-7)


def test_sharded_exchange_validates_before_enqueue(pkg):
    """ShardedAdamExchange.validate (engine.MappingEngine.iteration calls it before it enqueues
    anything) rejects what branch() cannot run: gradient rows changed after the exchange was built
    (its cached spans and the optimiser's shard state belong to the old buffers), the per-decoder
    backward (engine.merge False) and a trainable decoder other than the colour one."""
    from types import SimpleNamespace
    D = pkg.distributed

    class Eng(SimpleNamespace):
        def set_rows(self, rows, pad_rows=None):
            self.rows = rows
            self.pad_rows = self.pad_rows if pad_rows is None else pad_rows
            self.layout_gen += 1

    eng = Eng(merge=True, pad_rows=1, layout_gen=1, rows={})
    ex = D.ShardedAdamExchange(eng, optimizer=None, pack=lambda *a: None, unpack=lambda *a: None,
                               adam_slices=lambda *a: None)
    ex.validate(eng, ("grid_color",), ("color",))
    with pytest.raises(ValueError, match="only the colour decoder"):
        ex.validate(eng, ("grid_fine",), ("fine",))
    eng.merge = False
    with pytest.raises(ValueError, match="merged"):
        ex.validate(eng, ("grid_color",), ("color",))
    eng.merge = True
    eng.set_rows({})  # a new frustum selection: new buffers
    with pytest.raises(RuntimeError, match="rows changed"):
        ex.validate(eng, ("grid_color",), ("color",))
    with pytest.raises(ValueError, match="merged"):
        D.ShardedAdamExchange(Eng(merge=False, pad_rows=1, layout_gen=1, rows={}), optimizer=None)
