"""bench.py — ray-samples/s (fwd+bwd) of one NICE-SLAM mapping iteration, Replica room0 shape.

python bench.py [--gpus N --steps K --warmup W]   (N>1: launched by torch.distributed.run)

One step (the headline `value`) = one colour-stage iteration of the mapping engine that
Mapper.optimize_map's inner loop runs on (engine.MappingEngine.iteration: src/Mapper.py:391-519's
body), on synthetic room0 data resident in HBM (configs/Replica/room0.yaml bound, replica.yaml camera,
mapping.pixels=1000 over a 5-frame window, 32 stratified + 16 surface samples):
  pixel draws + rays (5 frames × 200, in the gather kernel) → inside-mask prefilter → sampler kernel →
  fused query kernel (middle+fine+colour decoders, 3 grid lookups) → loss kernel (compositing + mapping
  loss + their backward) → backward (one mask-only launch for the grid gradients ‖ the colour decoder's
  weight gradients) → [N>1: RCCL all-reduce of the frustum-row gradients] → Adam on the frustum rows +
  colour decoder — replayed from hipGraphs.
The reference entry points are timed in their own legs: "optimize_map" (Mapper.optimize_map per call,
60 iterations, BA off / on, against the bare engine's iterations of the same stage mix), "scene0000_ba"
(configs[2]: optimize_map with bundle adjustment, 5000 px) and "room0_slam_loop" (measured frames/s of
Tracker.track_frame every frame + Mapper.optimize_map every 5th frame).
Weak scaling: every rank maps its own 1000 rays; value = all ranks' ray-samples / max rank time.
"""
import argparse
import importlib
import json
import math
import os
import re
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# configs/Replica/room0.yaml:3, configs/Replica/replica.yaml cam + mapping, configs/nice_slam.yaml
# the next iteration's pixel gather + sampler run beside this iteration's render/backward
# (engine.MappingEngine.iteration(prefetch=True)); --no-prefetch for the strictly serial step
PREFETCH = True
# iterations per captured hipGraph, whatever --steps is (a replay starts only after the previous one has
# drained, ~20 us on MI355X: paid once per block), so runs of any length measure the same thing
GRAPH_BLOCK = 10
# gradient exchange of a ray-sharded run (N > 1): "allreduce" (SparseGradExchange: one all-reduce of the
# frustum rows + colour-decoder gradient after the backward, replicated Adam — one collective per
# iteration, on one stream) or "sharded" (reduce-scatter, Adam on the rank's shard, all-gather per
# backward branch: distributed.ShardedAdamExchange — four collectives on two communicators)
EXCHANGE = "allreduce"
# --force-exchange: a one-rank job issues the exchange's collectives anyway (RCCL identities), so the
# N > 1 code path — collectives captured in the hipGraph — runs on a one-GPU box
FORCE_EXCHANGE = False

ROOM0 = {
    "bound": [[-2.9, 8.9], [-3.2, 5.5], [-3.5, 3.3]], "bound_divisible": 0.32,
    "grid_len": {"coarse": 2.0, "middle": 0.32, "fine": 0.16, "color": 0.16},
    "H": 680, "W": 1200, "fx": 600.0, "fy": 600.0, "cx": 599.5, "cy": 339.5,
    "pixels": 1000, "window": 5, "n_strat": 32, "n_surf": 16, "w_color": 0.2,
    "lr": {"decoders": 0.005, "middle": 0.005, "fine": 0.005, "color": 0.005},
}
# configs[4] (BASELINE.json): synthetic 8 m cube, fine / colour grids 512^3 x 32 (16 GiB each), middle
# 256^3, 65536 pixels (4 frames x 16384) x 64 samples (48 stratified + 16 surface), colour stage
STRESS = dict(ROOM0, bound=[[0.0, 7.9]] * 3, bound_divisible=0.5,
              grid_len={"coarse": 2.0, "middle": 1 / 32, "fine": 1 / 64, "color": 1 / 64},
              pixels=65536, window=4, n_strat=48, n_surf=16)
# configs[3] (BASELINE.json): Apartment (configs/Apartment/apartment.yaml bound, Azure camera 720x1280),
# 5000 pixels per GPU (5 frames x 1000) x 48 samples, the full coarse -> middle -> fine -> colour
# hierarchy; the coarse mapper's iteration samples 32 stratified points without gt (Mapper.py:482-484)
APARTMENT = dict(ROOM0, bound=[[-5.8, 11.3], [-4.0, 4.5], [-7.9, 4.9]], bound_divisible=0.32,
                 H=720, W=1280, fx=607.4694213867188, fy=607.4534912109375, cx=636.9967041015625,
                 cy=369.2689514160156, pixels=5000, window=5, coarse=True)
# configs[2] (BASELINE.json): ScanNet scene0000 (configs/ScanNet/scene0000.yaml bound, scannet.yaml camera
# after crop_edge 10), 5000 pixels over a 5-frame window (4 keyframes + the current frame) x 48 samples,
# bundle adjustment of the 4 non-oldest cameras
SCENE0000 = dict(ROOM0, bound=[[-2.0, 11.0], [-2.0, 11.5], [-2.0, 5.5]], bound_divisible=0.32,
                 H=460, W=620, fx=577.590698, fy=578.729797, cx=308.905426, cy=232.683609, pixels=5000, window=5)
FLOP_FWD_PER_SAMPLE = 2 * (15479 + 20599 + 15575)   # SURVEY §8(a10) MACs, colour stage
FLOP_FINE_STAGE_PER_POINT = 2 * (15479 + 20599)          # fine stage: middle + fine decoders
BYTES_FWD_PER_SAMPLE = 3 * 1024                      # 3 trilinear lookups × 8 corners × 128 B
F32_PEAK_TFLOPS = 157.3                              # MI355X dense fp32 (MFMA = VALU rate)
HBM_PEAK_GBS = 8000.0
# Algorithmic work per ray-sample of each timed C-ABI launch of the colour-stage mapping
# iteration: (FLOPs, HBM bytes).  Forward: the three decoders' MACs and three
# 1024-B trilinear lookups.  Backward per decoder: the colour decoder (optimised) needs input and
# weight gradients = 2× its forward MACs; the frozen middle/fine decoders need input gradients
# only = 1× their MACs (mask-only backward, no recompute); each scatters one 8-corner gradient
# into its grid = 1024 B read + 1024 B written (float-atomic RMW).
KERNEL_WORK = {
    "query_fwd": (FLOP_FWD_PER_SAMPLE, BYTES_FWD_PER_SAMPLE),
    "query_bwd.color": (2 * 2 * 15575, 2048),
    # ABI v16: the colour decoder's weight gradients (dW = Σ cotangent ⊗ input: one MAC per weight per
    # sample; the recomputed cotangent chain, colour feature and Fourier terms are not counted)
    "query_bwd.color_wgrad": (2 * 15575, 0),
    "query_bwd.fine": (2 * 20599, 2048),
    "query_bwd.middle": (2 * 15479, 2048),
    # every decoder's mask-only backward (input gradients + grid scatter) as one launch (ABI v10
    # nslam_query_bwd_decoders): the fine / middle stages and the colour stage
    "query_bwd.middle+fine": (2 * 15479 + 2 * 20599, 2 * 2048),
    "query_bwd.middle+fine+color": (2 * 15479 + 2 * 20599 + 2 * 15575, 3 * 2048),
}
# The frozen decoders' mask-only backward launches are bound by their grid-gradient float atomics,
# not by HBM or MFMA: 8 corners x 32 channels x 4 B = 1024 added bytes per ray-sample against the
# chip-wide float-atomic rate of ~1.3 TB/s of added bytes (MI355X_MICROARCH.md, atomics table: every
# CU issuing, any footprint or contention).  Their roofline is stated against that ceiling.
ATOMIC_SPANS = {"query_bwd.fine": 1024, "query_bwd.middle": 1024, "query_bwd.middle+fine": 2048,
                "query_bwd.middle+fine+color": 3072}
ATOMIC_PEAK_GBS = 1300.0
# rocprofv3 kernel names behind each span (for the PMC traffic of profiles/*traffic*.json)
SPAN_KERNELS = {
    "query_fwd": ("k_query_fwd", "k_occ_combine"),
    "query_bwd.color": ("k_dec_bwd<3,", "k_color_wgrad", "k_slab_reduce"),
    "query_bwd.color_wgrad": ("k_color_wgrad", "k_slab_reduce"),
    "query_bwd.fine": ("k_dec_bwd<2,",),
    "query_bwd.middle": ("k_dec_bwd<1,",),
    "query_bwd.middle+fine": ("k_dec_bwd_multi<false>",),
    "query_bwd.middle+fine+color": ("k_dec_bwd_multi<false>",),
}
def _latest_profile(suffix):
    """profiles/rNN_<suffix> of the newest round that has one (the counters are collected per round)."""
    import glob
    found = sorted(glob.glob(os.path.join(REPO, "profiles", f"r[0-9][0-9]_{suffix}")))
    return found[-1] if found else os.path.join(REPO, "profiles", f"r04_{suffix}")


TRAFFIC_FILE = _latest_profile("traffic.json")
STRESS_TRAFFIC_FILE = _latest_profile("traffic_stress.json")
# SQ / GRBM counters of the same kernels (tools/gpu_counters.sh → tools/pmc_summary.py)
PMC_FILE = _latest_profile("room0_pmc.txt")
STRESS_PMC_FILE = _latest_profile("stress_pmc.txt")


def pmc_traffic(span, path=None):
    """HBM bytes per launch of `span` from the committed PMC summary (tools/traffic.py: separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over this bench, FETCH_SIZE doubled per the
    MI355X guide's gfx950 correction), or None when absent."""
    try:
        with open(path or TRAFFIC_FILE) as f:
            kern = json.load(f)["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    pats = SPAN_KERNELS.get(span, (span,))
    hits = [v["hbm_bytes_per_launch"] for k, v in kern.items() if any(k.startswith(p) for p in pats)]
    return sum(hits) if hits else None


def pmc_write_bytes(span, path=None):
    """WRITE_SIZE bytes per launch of `span` from the committed PMC summary (float atomics are
    counted exactly by WRITE_SIZE, MI355X guide), or None."""
    try:
        with open(path or TRAFFIC_FILE) as f:
            kern = json.load(f)["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    pats = SPAN_KERNELS.get(span, (span,))
    hits = [v["write_size_kib"] * 1024.0 for k, v in kern.items() if any(k.startswith(p) for p in pats)]
    return sum(hits) if hits else None


def pmc_counters(span, path=None):
    """The derived SQ counters (MFMA busy / SIMD-cycles, resident waves per SIMD, VALU issue, wait
    fractions, clock) and the average duration of the first rocprof kernel of `span` from a committed
    pmc_summary.py output, or None."""
    try:
        with open(path or PMC_FILE) as f:
            text = f.read()
    except OSError:
        return None
    pats = SPAN_KERNELS.get(span, (span,))
    for sec in text.split("== ")[1:]:
        head, _, body = sec.partition("\n")
        if not any(head.startswith(p) for p in pats):
            continue
        out = {"kernel": head.split("  (")[0], "file": os.path.relpath(path or PMC_FILE, REPO)}
        if "(avg " in head:
            out["avg_us"] = float(head.split("(avg ")[1].split(" us")[0])
        for line in body.splitlines():
            # "(name)   value   [(note)]": the derived figures of tools/pmc_summary.py
            mt = re.match(r"^\((.+?)\)\s+([-+0-9.eE]+)(?:\s+\((.*)\))?\s*$", line.strip())
            if mt:
                out[mt.group(1)] = float(mt.group(2))
                if mt.group(3):
                    out[mt.group(1) + " note"] = mt.group(3)
        return out
    return None


def pkg():
    return importlib.import_module("nice-slam_amd")


def enlarge_bound(cfg):
    """src/NICE_SLAM.py:145-150 (float32-rounded upper end)."""
    b = torch.tensor(cfg["bound"], dtype=torch.float64)
    cells = ((b[:, 1] - b[:, 0]) / cfg["bound_divisible"]).int() + 1
    b[:, 1] = (cells.float() * torch.tensor(cfg["bound_divisible"], dtype=torch.float32)).double() + b[:, 0]
    return b


def grid_shape(bound, glen):
    ext = bound[:, 1] - bound[:, 0]
    xyz = [int(v) for v in (ext / glen).tolist()]
    return [1, 32, xyz[2], xyz[1], xyz[0]]


def rot(yaw, pitch):
    cy, sy, cp, sp = math.cos(yaw), math.sin(yaw), math.cos(pitch), math.sin(pitch)
    Rz = torch.tensor([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]], dtype=torch.float64)
    Rx = torch.tensor([[1, 0, 0], [0, cp, -sp], [0, sp, cp]], dtype=torch.float64)
    return Rz @ Rx


class StepGraphs:
    """Whole mapping iterations as hipGraphs.  `block` (even) consecutive iterations form one
    graph, so the launch bubble between two graph replays (~20 us on MI355X: the next replay starts
    only after the previous one has drained) is paid once per block; two single-iteration graphs
    (one per ray-buffer parity of the prefetching engine) cover remainders.  run(k) executes exactly
    k iterations; finish() re-aligns the engine's host-side buffer parity (sync) with the device."""

    def __init__(self, fn, block=GRAPH_BLOCK, sync=None):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):
                fn()
        torch.cuda.current_stream().wait_stream(side)
        self.single = []
        # thread_local capture: RCCL's watchdog thread polls its work events while this thread captures
        # (global mode makes that poll fail the capture: hipErrorStreamCaptureUnsupported)
        for _ in range(2):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                fn()
            self.single.append(g)
        self.block = max(2, block - block % 2)
        self.blockg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.blockg, capture_error_mode="thread_local"):
            for _ in range(self.block):
                fn()
        self.par = 0  # device-side parity relative to the capture start
        self.sync = sync

    def run(self, k=1):
        while self.par == 0 and k >= self.block:
            self.blockg.replay()
            k -= self.block
        for _ in range(k):
            self.single[self.par].replay()
            self.par ^= 1

    def __call__(self):
        self.run(1)

    def finish(self):
        if self.par and self.sync is not None:
            self.sync()
        self.par = 0


def capture_step_graphs(fn, block=GRAPH_BLOCK, sync=None):
    """(StepGraphs, "hipgraph") for fn = one mapping iteration."""
    return StepGraphs(fn, block, sync), "hipgraph"


class Room0Scene:
    """Synthetic room0-shaped mapping workload (grids, decoders, 5 keyframes in HBM)."""

    def __init__(self, dev, rank=0, cfg=ROOM0, path="fused", device_init=False):
        P = pkg()
        self.cfg, self.dev = cfg, dev
        g = torch.Generator().manual_seed(2)
        self.bound = enlarge_bound(cfg)
        std = {"coarse": 0.01, "middle": 0.01, "fine": 1e-4, "color": 0.01}
        self.grids = {}
        self.coarse = bool(cfg.get("coarse"))
        for k in ("coarse",) * self.coarse + ("middle", "fine", "color"):
            # the coarse grid spans the bound enlarged x2 (NICE_SLAM.py:211-220, coarse_bound_enlarge)
            shp = grid_shape(self.bound, cfg["grid_len"][k] / (2.0 if k == "coarse" else 1.0))
            if device_init:  # stress grids (16 GiB): drawn on the device, channels-last directly
                gd = torch.Generator(device=dev).manual_seed(2 + len(self.grids))
                t = torch.empty(shp[0], shp[2], shp[3], shp[4], shp[1], device=dev).normal_(0.0, std[k], generator=gd)
                t = t.permute(0, 4, 1, 2, 3)
            else:
                t = (torch.randn(shp, generator=g) * std[k]).to(dev).contiguous(memory_format=torch.channels_last_3d)
            self.grids["grid_" + k] = t.requires_grad_(True)
        torch.manual_seed(3)
        self.nice = P.NICE(c_dim=32, coarse_grid_len=2.0, middle_grid_len=0.32, fine_grid_len=0.16,
                           color_grid_len=0.16, hidden_size=32, coarse=self.coarse)
        self.nice.set_bound(self.bound)
        self.nice = self.nice.to(dev)
        for d in (self.nice.middle_decoder, self.nice.fine_decoder):  # fix_fine; middle never optimised
            d.requires_grad_(False)
        self.renderer = P.Renderer({"rendering": {"N_samples": cfg["n_strat"], "N_surface": cfg["n_surf"],
                                                  "N_importance": 0, "lindisp": False, "perturb": 0.0},
                                    "occupancy": True}, None, _Slam(self.bound, cfg))
        # keyframes: poses at the room centre, seeded yaw/pitch; analytic depth to an inner box
        gk = torch.Generator().manual_seed(0)
        F = cfg["window"]
        ctr = self.bound.mean(1)
        self.c2w = torch.zeros(F, 3, 4, dtype=torch.float32)
        for f in range(F):
            yaw = float(torch.rand(1, generator=gk)) * 2 * math.pi
            pitch = (float(torch.rand(1, generator=gk)) - 0.5) * 0.6 + math.pi / 2
            self.c2w[f, :, :3] = rot(yaw, pitch).float()
            self.c2w[f, :, 3] = (ctr + (torch.rand(3, generator=gk, dtype=torch.float64) - 0.5) * 0.5).float()
        self.c2w = self.c2w.to(dev)
        H, W = cfg["H"], cfg["W"]
        jj, ii = torch.meshgrid(torch.arange(H, device=dev, dtype=torch.float32),
                                torch.arange(W, device=dev, dtype=torch.float32), indexing="ij")
        dirs = torch.stack([(ii - cfg["cx"]) / cfg["fx"], -(jj - cfg["cy"]) / cfg["fy"], -torch.ones_like(ii)], -1)
        inner = self.bound.clone()
        inner[:, 0] += 0.1 * (self.bound[:, 1] - self.bound[:, 0])
        inner[:, 1] -= 0.1 * (self.bound[:, 1] - self.bound[:, 0])
        inner = inner.to(dev)
        self.depth = torch.empty(F, H, W, device=dev)
        gd = torch.Generator(device=dev).manual_seed(1)
        for f in range(F):
            rd = (dirs.reshape(-1, 1, 3) * self.c2w[f, :, :3]).sum(-1).double()
            ro = self.c2w[f, :, 3].double().expand_as(rd)
            t = (inner[None] - ro[:, :, None]) / rd[:, :, None]
            d = t.max(2).values.min(1).values.float()
            d = d * (0.9 + 0.1 * torch.rand(d.shape, device=dev, generator=gd))
            d[torch.rand(d.shape, device=dev, generator=gd) < 0.05] = 0.0
            self.depth[f] = d.reshape(H, W)
        self.color = torch.rand(F, H, W, 3, device=dev, generator=gd)
        self.dirs = dirs.reshape(-1, 3)
        torch.cuda.manual_seed(1000 + rank)  # pixel draws use the (graph-safe) default generator
        self.bound_dev = self.bound.to(dev)
        self.frames = [(self.depth[f], self.color[f], self.c2w[f]) for f in range(F)]
        # frustum_feature_selection (Mapper.py:314-333): voxels seen by the current frame (frame 0)
        self.rows = {}
        for k in ("grid_middle", "grid_fine", "grid_color"):
            m = P.mapper.frustum_mask(self.c2w[0], k, self.grids[k].shape[2:], self.depth[0], self.bound, H, W,
                                      cfg["fx"], cfg["fy"], cfg["cx"], cfg["cy"])
            self.rows[k] = P.engine.frustum_rows(m)
        self.path = path
        self.kept = torch.zeros(1, dtype=torch.int64, device=dev)
        self.rank = rank
        if path == "fused":
            for t in self.grids.values():
                t.requires_grad_(False)
            # grid gradients accumulate only on the frustum-selected rows Adam optimises (compact)
            self.engine = P.engine.MappingEngine(self.nice, self.grids, self.bound, cfg["n_strat"], cfg["n_surf"],
                                                 w_color=cfg["w_color"], device=dev, rows=self.rows)
            self.opt = P.ops.FusedAdam(
                [{"params": [self.engine.decs["color"].param], "lr": cfg["lr"]["decoders"]}] +
                ([{"params": [self.grids["grid_coarse"]], "lr": cfg["lr"]["middle"]}] if self.coarse else []) +
                [{"params": [self.grids[k]], "lr": cfg["lr"][k[5:]], "rows": self.rows[k]}
                 for k in ("grid_middle", "grid_fine", "grid_color")])
            # ray-sharded: exchange only the frustum rows Adam reads (+ colour-decoder grads) — by default
            # reduce-scatter, Adam on this rank's shard, all-gather, per backward branch
            # (distributed.ShardedAdamExchange); --exchange allreduce: one all-reduce, replicated Adam
            world = int(os.environ.get("WORLD_SIZE", "1"))
            if (world > 1 or FORCE_EXCHANGE) and EXCHANGE == "sharded":
                self.exchange = P.distributed.ShardedAdamExchange(self.engine, self.opt,
                                                                  force_collectives=FORCE_EXCHANGE)
            else:
                self.exchange = P.distributed.SparseGradExchange(self.engine, self.rows,
                                                                 force_collectives=FORCE_EXCHANGE)
        else:
            params = [{"params": list(self.nice.color_decoder.parameters()), "lr": cfg["lr"]["decoders"]},
                      {"params": [self.grids["grid_middle"]], "lr": cfg["lr"]["middle"]},
                      {"params": [self.grids["grid_fine"]], "lr": cfg["lr"]["fine"]},
                      {"params": [self.grids["grid_color"]], "lr": cfg["lr"]["color"]}]
            self.opt = torch.optim.Adam(params, fused=True, capturable=True)

    def sample_batch(self):
        """get_samples over the window (Mapper.py:437-467): 200 random pixels per frame."""
        cfg = self.cfg
        F, H, W = cfg["window"], cfg["H"], cfg["W"]
        n = cfg["pixels"] // F
        idx = torch.randint(H * W, (F, n), device=self.dev)
        depth = torch.gather(self.depth.reshape(F, -1), 1, idx).reshape(-1)
        color = torch.gather(self.color.reshape(F, -1, 3), 1, idx[..., None].expand(F, n, 3)).reshape(-1, 3)
        d = self.dirs[idx]                                              # [F, n, 3]
        rays_d = torch.einsum("fnk,fjk->fnj", d, self.c2w[:, :, :3]).reshape(-1, 3)
        rays_o = self.c2w[:, None, :, 3].expand(F, n, 3).reshape(-1, 3)
        return rays_o, rays_d, depth, color

    def step(self, stage="color", sharded=False):
        """One colour-stage mapping iteration, no host synchronisation (hipGraph-capturable).
        Pixels are drawn inside the gather kernel (uniform over the image, like select_uv) and
        the gather kernel adds the kept-ray count into self.kept: kept ray-samples over a run =
        self.kept × samples per ray, read once after the timed region."""
        if self.path != "fused":
            return self.step_autograd(stage, sharded)
        cfg = self.cfg
        F, H, W = cfg["window"], cfg["H"], cfg["W"]
        n = cfg["pixels"] // F
        # ray-sharded: one global batch of pixels * world draws (same seed on every rank), each rank
        # gathering its slice; the gather kernel also yields the global batch's max(gt_depth), so
        # the only collective of the iteration is the gradient exchange
        world = int(os.environ.get("WORLD_SIZE", "1")) if sharded else 1
        self.engine.iteration(
            stage, self.frames, None, n, (H, W), (cfg["fx"], cfg["fy"], cfg["cx"], cfg["cy"]), self.opt,
            trainable_decoders=("color",), exchange=self.exchange if sharded else None, n_kept=self.kept,
            seed=1000, world=world, rank=self.rank if sharded else 0, prefetch=PREFETCH)

    def flip_parity(self):
        """The prefetching engine's host-side ray-buffer parity, after an odd number of replayed
        iterations (StepGraphs.finish)."""
        if self.path == "fused":
            self.engine._parity ^= 1

    def step_autograd(self, stage="color", sharded=False):
        """The same iteration through the autograd drop-in path (dense Adam, torch glue ops).

        The inside-mask prefilter (Mapper.py:469-481) removes rays; here they stay in the batch
        with zero loss weight (their gradients are exactly zero) and the sampler's batch-global
        max(gt_depth) is taken over the kept rays only — the same maths without a host-side
        compaction.  Returns the number of kept ray-samples (device tensor).
        """
        cfg = self.cfg
        D = pkg().distributed
        self.opt.zero_grad(set_to_none=True)
        rays_o, rays_d, gt_depth, gt_color = self.sample_batch()
        with torch.no_grad():
            t = (self.bound_dev[None] - rays_o[..., None].double()) / rays_d[..., None].double()
            keep = t.max(2).values.min(1).values >= gt_depth
            gmax = torch.where(keep, gt_depth, torch.full_like(gt_depth, float("-inf"))).max().reshape(1)
            if sharded:
                gmax = D.global_max(gmax)
        depth, unc, color = self.renderer.render_batch_ray(self.grids, self.nice, rays_d, rays_o, self.dev, stage,
                                                           gt_depth=gt_depth, gt_max=gmax)
        m = keep & (gt_depth > 0)
        loss = torch.where(m, torch.abs(gt_depth - depth), torch.zeros_like(depth)).sum()
        if stage == "color":
            cl = torch.where(keep[:, None], torch.abs(gt_color - color), torch.zeros_like(color)).sum()
            loss = loss + cfg["w_color"] * cl
        loss.backward()
        if sharded:
            D.allreduce_grads(D.optimizer_params(self.opt))
        self.opt.step()
        self.kept += keep.sum()


class _Slam:
    def __init__(self, bound, cfg):
        self.nice, self.bound = True, bound
        self.H, self.W, self.fx, self.fy, self.cx, self.cy = cfg["H"], cfg["W"], cfg["fx"], cfg["fy"], cfg["cx"], cfg["cy"]


def cpu_model():
    """The host CPU's model name (lscpu's 'Model name', from /proc/cpuinfo)."""
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(scene, budget_s=20.0, reps=5):
    """The oracle (torch CPU restatement, oracle/nslam_oracle.py) on the same workload, host cores:
    one warm-up iteration, then `reps` timed samples of a few iterations each (about budget_s in
    all); value = the median sample's ray-samples/s (BASELINE.md's warm-up + median-of-5 plan)."""
    from oracle import nslam_oracle as orc
    threads = torch.get_num_threads()
    bound = scene.bound
    grids = {k: v.detach().cpu().contiguous().requires_grad_(True) for k, v in scene.grids.items()}
    sd = {k: v.detach().cpu() for k, v in scene.nice.state_dict().items()}
    for k in list(sd):
        if k.startswith("color_decoder."):
            sd[k] = sd[k].clone().requires_grad_(True)
    opt = torch.optim.Adam([v for k, v in sd.items() if v.requires_grad] + list(grids.values()), lr=0.005)

    def iteration():
        ro, rd, gt, gc = (x.cpu() for x in scene.sample_batch())
        keep = orc.inside_mask(ro, rd, gt, bound)
        ro, rd, gt, gc = ro[keep], rd[keep], gt[keep], gc[keep]
        opt.zero_grad()
        d, v, c = orc.render_batch_ray(sd, grids, rd, ro, "color", bound, gt)
        orc.mapper_loss(d, c, gt, gc, "color").backward()
        opt.step()
        return ro.shape[0] * 48

    t0 = time.perf_counter()
    iteration()                                        # warm-up
    per_iter = time.perf_counter() - t0
    n = max(1, int(budget_s / reps / max(per_iter, 1e-3)))
    rates, tot_iters, tot_s = [], 0, 0.0
    for _ in range(reps):
        samples, t0 = 0, time.perf_counter()
        for _ in range(n):
            samples += iteration()
        dt = time.perf_counter() - t0
        rates.append(samples / dt)
        tot_iters, tot_s = tot_iters + n, tot_s + dt
    rates.sort()
    return {"value": rates[reps // 2], "unit": "ray-samples/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "samples_per_s_all": rates,
            "sample": f"median of {reps} samples of {n} colour-stage mapping iterations each (1000 rays x 48 "
                      f"samples, fwd+bwd+Adam) after 1 warm-up, oracle/nslam_oracle.py on {threads} host threads "
                      f"({cpu_model()}), {tot_iters} iterations in {tot_s:.1f} s"}


def stress_grid_query(dev, side=512, rays=65536, samples=64, reps=10):
    """The grid-query kernel alone at BASELINE.json's HBM-roofline stress shape:
    one fine grid of side³ voxels × 32 ch fp32 (512³: 16 GiB, far beyond the 256 MiB Infinity
    Cache), 65536 rays × 64 samples through it (random origins and directions in the unit cube,
    samples evenly spaced to the exit), nslam_grid_sample_fwd timed with HIP events on its stream.
    Algorithmic bytes per point: 8 corners × 128 B read + 128 B feature row written + 12 B coords."""
    P = pkg()
    g = torch.Generator(device=dev).manual_seed(7)
    grid = torch.empty(1, side, side, side, 32, device=dev).normal_(0.0, 1e-4, generator=g).permute(0, 4, 1, 2, 3)
    o = torch.rand(rays, 3, device=dev, generator=g) * 2 - 1
    d = torch.randn(rays, 3, device=dev, generator=g)
    d = d / d.norm(dim=1, keepdim=True)
    t = torch.maximum((1 - o) / d, (-1 - o) / d).min(1).values              # exit distance (>0)
    z = torch.linspace(0.0, 1.0, samples, device=dev)[None] * t[:, None]
    coords = (o[:, None] + d[:, None] * z[..., None]).clamp_(-1, 1).reshape(-1, 3).contiguous()
    n = coords.shape[0]
    out = torch.empty(n, 32, device=dev)
    P.ops.grid_sample_fwd(grid, coords, out)                                  # warm-up
    P.ops.TIMER = P.ops.KernelTimer()
    for _ in range(reps):
        P.ops.grid_sample_fwd(grid, coords, out)
    tm = P.ops.TIMER.summary()["grid_fwd"]
    P.ops.TIMER = None
    bpp = 8 * 128 + 128 + 12
    achieved = n * bpp / (tm["avg_ms"] * 1e-3) / 1e9
    del grid, out, coords
    torch.cuda.empty_cache()
    traffic = pmc_traffic("k_grid_fwd", STRESS_TRAFFIC_FILE)
    # frac on the PMC-counted HBM bytes (FETCH_SIZE x2 + WRITE_SIZE per launch) when the committed
    # summary has them: the algorithmic count includes L2 / MALL reuse between a ray's samples
    counted = traffic / (tm["avg_ms"] * 1e-3) / 1e9 if traffic else None
    return {"kernel": "k_grid_fwd (nslam_grid_sample_fwd)", "bound": "hbm",
            "achieved": counted if counted else achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": (counted if counted else achieved) / HBM_PEAK_GBS, "frac_basis": "pmc" if counted else "algorithmic",
            "achieved_algorithmic": achieved, "frac_algorithmic": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "avg_launch_ms": tm["avg_ms"], "points": n, "bytes_per_point": bpp,
            "workload": f"grid [1,32,{side},{side},{side}] fp32 channels-last (16 GiB), {rays} rays x {samples} "
                        "samples, random rays through the cube"}


def stress_iteration(dev, steps=10):
    """configs[4] as a whole mapping iteration on the fused engine (SURVEY §8(d) stress row): the
    colour-stage iteration of the room0 bench at the stress shape — 8 m cube, fine / colour grids
    512^3 x 32 (16 GiB each), middle 256^3, 65536 pixels over 4 frames x 64 samples, frustum-masked
    Adam — replayed in a hipGraph.  Per-kernel HIP-event spans come from extra eager iterations;
    the forward's 3 trilinear lookups (3 KiB per sample) are priced against the HBM roof, its FLOPs
    against the fp32 MFMA roof."""
    global PREFETCH
    scene = Room0Scene(dev, 0, cfg=dict(STRESS), path="fused", device_init=True)
    P = pkg()
    if os.environ.get("NSLAM_BENCH_EAGER"):  # counter passes: every kernel alone on the chip
        scene.engine.concurrent = False
        PREFETCH = False
    for _ in range(2):
        scene.step()
    torch.cuda.synchronize()
    if os.environ.get("NSLAM_BENCH_EAGER"):  # PMC passes (tools/gpu_traffic_stress.sh): per-dispatch counters
        g, mode = None, "eager"
    else:
        g, mode = capture_step_graphs(scene.step, block=2, sync=scene.flip_parity)
        g.run(2)
    torch.cuda.synchronize()
    scene.kept.zero_()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if g is not None:
        g.run(steps)
    else:
        for _ in range(steps):
            scene.step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if g is not None:
        g.finish()
    samples = int(scene.kept) * (STRESS["n_strat"] + STRESS["n_surf"])
    timers = span_timers(scene, 3)
    pts = samples / steps
    fwd = timers["query_fwd"]["avg_ms"] * 1e-3
    rows = {k: int(v.numel()) for k, v in scene.rows.items()}
    out = {"value": samples / dt, "unit": "ray-samples/s", "ms_per_iteration": dt / steps * 1e3, "steps": steps,
           "launch_mode": mode, "ray_samples_per_iteration": pts,
           "kernels_ms": {k: round(v["avg_ms"], 4) for k, v in timers.items()},
           "query_fwd_roofline": kernel_roofline("query_fwd", timers["query_fwd"]["avg_ms"], pts, STRESS_TRAFFIC_FILE,
                                                 STRESS_PMC_FILE),
           "kernel_rooflines": {k: kernel_roofline(k, v["avg_ms"], pts, STRESS_TRAFFIC_FILE, STRESS_PMC_FILE)
                                for k, v in timers.items() if k in KERNEL_WORK},
           "query_fwd_gather_gbs": pts * BYTES_FWD_PER_SAMPLE / fwd / 1e9,
           "query_fwd_gather_hbm_frac": pts * BYTES_FWD_PER_SAMPLE / fwd / 1e9 / HBM_PEAK_GBS,
           "frustum_rows": rows,
           "workload": "configs[4]: 8 m cube, grids middle 256^3 / fine 512^3 / colour 512^3 x 32 fp32 "
                       "channels-last, 65536 pixels (4 frames x 16384) x 64 samples, colour stage, Adam on "
                       "the frustum rows"}
    del scene
    torch.cuda.empty_cache()
    return out


def bulk_queries(scene, res=256, reps=2):
    """Forward-only bulk queries through the drop-in API on the same kernels:
    Mesher.get_mesh's grid evaluation (Mesher.py:281-319,382-433: res³ points over the bound in
    Renderer.points_batch_size = 500k chunks, fine stage for occupancy and colour stage for the
    vertex colours) and Renderer.render_img at room0 size (Renderer.py:200-255: H×W rays × 48
    samples in 100k-ray batches, with the frame's depth as gt).  Timed with events on the stream."""
    dev = scene.dev
    nice, grids, r = scene.nice, scene.grids, scene.renderer
    b = scene.bound
    ax = [torch.linspace(float(b[k, 0]), float(b[k, 1]), res, dtype=torch.float64, device=dev) for k in range(3)]
    pts = torch.stack(torch.meshgrid(*ax, indexing="ij"), -1).reshape(-1, 3)
    out = {}

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    with torch.no_grad():
        for stage, fl in (("fine", FLOP_FINE_STAGE_PER_POINT), ("color", FLOP_FWD_PER_SAMPLE)):
            def mesh():
                for i in range(0, pts.shape[0], r.points_batch_size):
                    r.eval_points(pts[i:i + r.points_batch_size], nice, grids, stage, dev)
            ms = timed(mesh)
            n = pts.shape[0]
            tf = n * fl / (ms * 1e-3) / 1e12
            out["mesh_eval_" + stage] = {
                "points": n, "ms": ms, "points_per_s": n / (ms * 1e-3), "flop_per_point": fl,
                "achieved_tflops": tf, "frac_mfma_peak": tf / F32_PEAK_TFLOPS,
                "workload": f"{res}^3 grid points over the room0 bound, eval_points in 500k-point chunks"}
        c2w = scene.c2w[0]
        ms = timed(lambda: r.render_img(grids, nice, c2w, dev, "color", gt_depth=scene.depth[0]))
        n = scene.cfg["H"] * scene.cfg["W"] * (scene.cfg["n_strat"] + scene.cfg["n_surf"])
        out["render_img"] = {"ms_per_image": ms, "ray_samples_per_s": n / (ms * 1e-3),
                             "workload": f"{scene.cfg['H']}x{scene.cfg['W']} rays x 48 samples, colour stage, "
                                         "100k-ray batches, gt depth"}
    del pts
    torch.cuda.empty_cache()
    return out


def frame_io(dev, n=6, n_prefetch=128, workers=8):
    """Frame source: Replica-format frames at room0 size (680×1200 JPEG colour,
    16-bit PNG depth, traj.txt) written to a temp folder, then read through datasets.Replica onto
    the device — decode + H2D per frame, float64 colour (the reference's, datasets.py:91) vs the
    float32 colour the engine keeps resident; and through Replica.prefetch (the reference's
    DataLoader worker, Tracker.py:64-65: `workers` decode processes, pinned buffers, H2D on a side
    stream) over `n_prefetch` frames."""
    import tempfile

    import numpy as np
    from PIL import Image
    P = pkg()
    H, W = ROOM0["H"], ROOM0["W"]
    rng = np.random.default_rng(0)
    out = {}
    with tempfile.TemporaryDirectory() as d:
        os.makedirs(os.path.join(d, "results"))
        yy, xx = np.mgrid[0:H, 0:W]
        nf = max(n, 16)  # files on disk; the read-ahead pass cycles through them
        for i in range(nf):  # smooth synthetic content (JPEG cost like a real frame, not noise)
            img = np.stack([(xx * 255 // W + 20 * i) % 256, yy * 255 // H, (xx + yy) % 256], -1).astype(np.uint8)
            Image.fromarray(img).save(os.path.join(d, f"results/frame{i:06d}.jpg"), quality=95)
            Image.fromarray(rng.integers(5000, 30000, (H, W)).astype(np.uint16)).save(
                os.path.join(d, f"results/depth{i:06d}.png"))
        with open(os.path.join(d, "traj.txt"), "w") as f:
            for _ in range(nf):
                f.write(" ".join(str(v) for v in np.eye(4).ravel()) + "\n")
        cfg = {"dataset": "replica", "data": {"input_folder": d},
               "cam": {"H": H, "W": W, "fx": 600.0, "fy": 600.0, "cx": 599.5, "cy": 339.5,
                       "png_depth_scale": 6553.5, "crop_edge": 0}}
        for name, cd in (("f64", torch.float64), ("f32", torch.float32)):
            ds = P.get_dataset(cfg, None, 1.0, device=dev, color_dtype=cd)
            ds[0]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(n):
                ds[i]
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / n
            out["color_" + name] = {"ms_per_frame": dt * 1e3, "frames_per_s": 1.0 / dt,
                                    "device_bytes_per_frame": H * W * (3 * (8 if cd == torch.float64 else 4) + 4),
                                    "h2d_bytes_per_frame": H * W * (3 + 4)}
            # read-ahead: worker processes decode, H2D on a side stream (a consumer would render meanwhile)
            ds = P.get_dataset(cfg, None, 1.0, device=dev, color_dtype=cd)
            torch.cuda.synchronize()
            t_start = time.perf_counter()
            k, t0 = -1, None
            for _ in ds.prefetch([i % nf for i in range(n_prefetch)], workers=workers, ahead=2 * workers):
                if t0 is None:  # steady state: from the first frame handed out (workers started)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                k += 1
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            dt = (t1 - t0) / max(k, 1)
            out["prefetch_" + name] = {"ms_per_frame": dt * 1e3, "frames_per_s": 1.0 / dt, "frames": k,
                                       "workers": workers, "startup_ms": (t0 - t_start) * 1e3,
                                       "frames_per_s_incl_startup": (k + 1) / (t1 - t_start)}
    out["workload"] = (f"{n} Replica-format frames {H}x{W} (JPEG q95 colour, 16-bit PNG depth), Pillow decode + H2D, "
                       f"one by one (dataset[i]) and {n_prefetch} through dataset.prefetch ({workers} workers)")
    return out


def reference_gpu_baseline(scene, budget_s=4.0):
    """The reference's PyTorch path ON THE GPU, for the ≥10x target of BASELINE.json: the oracle's
    restatement of Renderer.render_batch_ray + Mapper loss (the same torch ops the reference issues:
    F.grid_sample, nn.Linear, cumprod, autograd, torch.optim.Adam) on the same device-resident
    workload.  It omits the reference's per-iteration masked-grid copies (Mapper.py:394-401,
    511-519), so it is if anything faster than the reference."""
    from oracle import nslam_oracle as orc
    dev = scene.dev
    bound = scene.bound.to(dev)
    grids = {k: v.detach().clone().requires_grad_(True) for k, v in scene.grids.items()}
    sd = {k: v.detach().clone() for k, v in scene.nice.state_dict().items()}
    for k in list(sd):
        if k.startswith("color_decoder."):
            sd[k].requires_grad_(True)
    opt = torch.optim.Adam([v for v in sd.values() if v.requires_grad] + list(grids.values()), lr=0.005)
    samples, iters = 0, 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while iters < 3 or (time.perf_counter() - t0 < budget_s and iters < 400):
        if iters == 2:  # two warm-up iterations
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        ro, rd, gt, gc = scene.sample_batch()
        keep = orc.inside_mask(ro, rd, gt, bound)
        ro, rd, gt, gc = ro[keep], rd[keep], gt[keep], gc[keep]
        opt.zero_grad()
        d, v, c = orc.render_batch_ray(sd, grids, rd, ro, "color", bound, gt)
        orc.mapper_loss(d, c, gt, gc, "color").backward()
        opt.step()
        if iters >= 2:
            samples += ro.shape[0] * 48
        iters += 1
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"value": samples / dt, "unit": "ray-samples/s", "ms_per_step": dt / (iters - 2) * 1e3,
            "sample": f"{iters - 2} colour-stage mapping iterations after 2 warm-ups: oracle/nslam_oracle.py "
                      "(torch ops of the reference path) on the GPU, eager"}


def kernel_roofline(name, avg_ms, pts, traffic_path=None, pmc_path=None):
    """Roofline of one timed launch: algorithmic FLOPs and bytes (KERNEL_WORK × ray-samples per
    launch) over its HIP-event average; the bound is whichever roof (fp32 MFMA, HBM) the
    algorithmic work would hit first — or, for the frozen decoders' mask-only backward, the
    chip-wide float-atomic rate its grid-gradient scatter is bound by (ATOMIC_SPANS)."""
    fl, by = KERNEL_WORK[name]
    t = avg_ms * 1e-3
    tflops, gbs = pts * fl / t / 1e12, pts * by / t / 1e9
    mfma = fl / (F32_PEAK_TFLOPS * 1e12) >= by / (HBM_PEAK_GBS * 1e9)
    achieved, peak, unit = (tflops, F32_PEAK_TFLOPS, "TFLOP/s") if mfma else (gbs, HBM_PEAK_GBS, "GB/s")
    bound = "mfma" if mfma else "hbm"
    extra = {}
    if name in ATOMIC_SPANS:
        # the atomic bytes the kernel really issues: PMC WRITE_SIZE (exact for float atomics) when the
        # committed summary has it — the scatter walk merges runs of samples, so far fewer than the
        # 1024 B per sample and grid before merging; else that algorithmic count
        counted = pmc_write_bytes(name, traffic_path or TRAFFIC_FILE)
        abytes = counted if counted else pts * ATOMIC_SPANS[name]
        bound, achieved, peak, unit = "atomic", abytes / t / 1e9, ATOMIC_PEAK_GBS, "GB/s"
        extra = {"atomic_bytes_per_sample_unmerged": ATOMIC_SPANS[name],
                 "atomic_bytes_per_launch": abytes, "atomic_basis": "pmc WRITE_SIZE" if counted else "algorithmic",
                 "atomic_note": "float-atomic adds into the grid gradient against ~1.3 TB/s of added bytes chip-wide "
                                "(MI355X_MICROARCH.md atomics table); well under it, these mask-only kernels are "
                                "latency-bound; mfma_frac = input-gradient FLOPs vs fp32 peak",
                 "mfma_frac": tflops / F32_PEAK_TFLOPS}
    tp = traffic_path or TRAFFIC_FILE
    return {"kernel": name, "bound": bound, "achieved": achieved, "peak": peak, "unit": unit,
            "frac": achieved / peak, "traffic": pmc_traffic(name, tp), "avg_launch_ms": avg_ms,
            "ray_samples_per_launch": pts, "flop_per_sample": fl, "bytes_per_sample": by, **extra,
            # the HIP-event span brackets these rocprofv3 kernels back to back: compare its average
            # with the SUM of their average durations in the rocprof summary under profiles/
            "rocprof_kernels": list(SPAN_KERNELS.get(name, ())),
            "traffic_note": "HBM bytes per launch: rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE, "
                            + os.path.relpath(tp, REPO),
            # the counters behind the bound: SQ_VALU_MFMA_BUSY_CYCLES etc. of the span's first kernel
            "pmc": pmc_counters(name, pmc_path)}


def span_timers(scene, steps, sharded=False):
    """HIP-event spans of every C-ABI launch over `steps` extra eager iterations, with the backward
    branches serialised (engine.concurrent = False): each span is then one kernel (or one kernel +
    its slab reduction) alone on the chip, the duration its roofline is priced on.  The timed
    iterations (the headline value) run the branches concurrently."""
    P = pkg()
    eng = getattr(scene, "engine", None)
    conc = eng.concurrent if eng is not None else None
    if eng is not None:
        eng.concurrent = False
    P.ops.TIMER = P.ops.KernelTimer()
    try:
        for _ in range(steps):
            scene.step(sharded=sharded)
        return P.ops.TIMER.summary()
    finally:
        P.ops.TIMER = None
        if eng is not None:
            eng.concurrent = conc


def graph_time(scene, fn, reps):
    """(ms per call, launch mode) of fn = one iteration, captured in hipGraphs and replayed `reps`
    times after 3 eager and 10 replayed warm-ups."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    try:  # graph blocks of GRAPH_BLOCK iterations, as the headline leg
        g, mode = capture_step_graphs(fn, sync=scene.flip_parity)
        run = g.run
    except Exception:  # pragma: no cover - eager fallback
        g, mode = None, "eager"

        def run(k):
            for _ in range(k):
                fn()
    run(10)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(reps)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps * 1e3
    if g is not None:
        g.finish()
    return dt, mode


def apartment_iterations(dev, reps=50):
    """configs[3] on one GPU (its per-rank share of the 8-GPU job): Apartment bound and camera, 5000
    pixels over a 5-frame window, every stage of the hierarchy as one fused-engine mapping iteration
    replayed in a hipGraph — the coarse mapper's iteration (Mapper.py:403-404,482-484: stage
    'coarse', no gt in the sampler so 32 stratified samples, depth loss, dense coarse-grid Adam) and
    the fine mapper's middle / fine / colour iterations (frustum-masked grids, colour decoder)."""
    scene = Room0Scene(dev, 0, cfg=dict(APARTMENT), path="fused")
    cfg = scene.cfg
    out = {"ms_per_iteration": {}, "ray_samples_per_s": {}}
    for stage in ("coarse", "middle", "fine", "color"):
        ms, mode = graph_time(scene, lambda: scene.step(stage=stage), reps)
        out["ms_per_iteration"]["map_" + stage] = round(ms, 4)
        spr = cfg["n_strat"] if stage == "coarse" else cfg["n_strat"] + cfg["n_surf"]
        # kept rays per iteration from one extra eager iteration's count
        scene.kept.zero_()
        scene.step(stage=stage)
        torch.cuda.synchronize()
        out["ray_samples_per_s"]["map_" + stage] = int(scene.kept) * spr / (ms * 1e-3)
    out["launch_mode"] = mode
    out["grids"] = {k: list(v.shape) for k, v in scene.grids.items()}
    # the frustum rows Adam reads = the per-iteration exchange payload of a ray-sharded job
    out["frustum_rows"] = {k: int(v.numel()) for k, v in scene.rows.items()}
    out["workload"] = ("configs[3] Apartment, 1 GPU: 5000 pixels (5 frames x 1000) per iteration; coarse 32 samples "
                       "(no gt), middle/fine/colour 48 samples, frustum-masked Adam (coarse grid dense)")
    del scene
    torch.cuda.empty_cache()
    return out


def room0_frame_rate(scene, reps=100):
    """frames/s on Replica room0 (BASELINE metric) from measured iteration times:
    per frame 10 tracking iterations × 200 pixels (replica.yaml tracking, edges 100 px) and 12
    mapping iterations × 1000 pixels (60 iterations every 5 frames, stage split middle 25 / fine 12
    / colour 23 of 60: Mapper.py:403-419).  Each iteration type is captured in a hipGraph and
    replayed `reps` times.  'sequential' = tracker and mapper on one stream back to back (a lower
    bound; the reference runs them as concurrent processes)."""
    P = pkg()
    cfg = scene.cfg
    H, W = cfg["H"], cfg["W"]

    def timed(fn):
        return graph_time(scene, fn, reps)

    ms = {}
    for stage in ("middle", "fine", "color"):
        ms["map_" + stage], _ = timed(lambda: scene.step(stage=stage))
    import copy
    te = P.engine.TrackingEngine(copy.deepcopy(scene.nice), scene.grids, scene.bound, cfg["n_strat"], cfg["n_surf"],
                                 (H, W), (cfg["fx"], cfg["fy"], cfg["cx"], cfg["cy"]), ignore_edge=(100, 100),
                                 w_color=0.5, handle_dynamic=True, use_color=True, device=scene.dev)
    cam = P.common.get_tensor_from_camera(scene.c2w[0]).to(scene.dev).requires_grad_(True)
    opt = P.ops.FusedAdam([{"params": [cam], "lr": 0.001}])
    nwin = te.n_window()

    def track():
        pix = torch.randint(nwin, (200,), device=scene.dev)
        te.iteration(cam, scene.depth[0], scene.color[0], pix, opt)

    ms["track"], tmode = timed(track)
    t_map = (25 * ms["map_middle"] + 12 * ms["map_fine"] + 23 * ms["map_color"]) / 60.0
    t_frame = 10 * ms["track"] + 12 * t_map
    return {"frames_per_s": 1e3 / t_frame, "frames_per_s_concurrent": 1e3 / max(10 * ms["track"], 12 * t_map),
            "ms_per_iteration": {k: round(v, 4) for k, v in ms.items()}, "tracking_launch_mode": tmode,
            "note": "sequential: 10 tracking + 12 mapping iterations per frame on one GPU stream; concurrent: "
                    "tracker and mapper overlapped as the reference's processes (max of the two)"}


def nice_slam_cfg(cfg, tracking_edge=100):
    """The reference's configs/nice_slam.yaml tracking / mapping keys with a scene's camera and pixel
    counts (configs/Replica/replica.yaml, configs/ScanNet/scannet.yaml): what Tracker / Mapper read."""
    st = {"coarse": {"decoders_lr": 0.0, "coarse_lr": 0.001, "middle_lr": 0.0, "fine_lr": 0.0, "color_lr": 0.0},
          "middle": {"decoders_lr": 0.0, "coarse_lr": 0.0, "middle_lr": 0.1, "fine_lr": 0.0, "color_lr": 0.0},
          "fine": {"decoders_lr": 0.0, "coarse_lr": 0.0, "middle_lr": 0.005, "fine_lr": 0.005, "color_lr": 0.0},
          "color": {"decoders_lr": 0.005, "coarse_lr": 0.0, "middle_lr": 0.005, "fine_lr": 0.005, "color_lr": 0.005}}
    return {"coarse": False, "occupancy": True, "scale": 1,
            "rendering": {"N_samples": cfg["n_strat"], "N_surface": cfg["n_surf"], "N_importance": 0, "lindisp": False,
                          "perturb": 0.0},
            "tracking": {"lr": 0.001, "device": "cuda:0", "iters": 10, "gt_camera": False, "pixels": 200,
                         "seperate_LR": False, "w_color_loss": 0.5, "ignore_edge_W": tracking_edge,
                         "ignore_edge_H": tracking_edge, "handle_dynamic": True, "use_color_in_tracking": True,
                         "const_speed_assumption": True},
            "mapping": {"device": "cuda:0", "fix_fine": True, "BA_cam_lr": 0.001, "fix_color": False,
                        "pixels": cfg["pixels"], "iters": 60, "w_color_loss": cfg["w_color"], "fine_iter_ratio": 0.6,
                        "middle_iter_ratio": 0.4, "mapping_window_size": cfg["window"],
                        "frustum_feature_selection": True, "keyframe_selection_method": "overlap", "stage": st}}


def slam_state(scene):
    """What Tracker / Mapper read from the reference's NICE_SLAM object, over a scene's tensors."""
    from types import SimpleNamespace
    cfg = scene.cfg
    return SimpleNamespace(nice=True, bound=scene.bound, H=cfg["H"], W=cfg["W"], fx=cfg["fx"], fy=cfg["fy"],
                           cx=cfg["cx"], cy=cfg["cy"], shared_decoders=scene.nice, shared_c=scene.grids,
                           renderer=scene.renderer, estimate_c2w_list=torch.zeros(4, 4, 4),
                           gt_c2w_list=torch.zeros(4, 4, 4), mapping_idx=torch.zeros(1).int())


def _pose4(c2w):
    return torch.cat([c2w, torch.tensor([[0, 0, 0, 1.0]], device=c2w.device)], 0)


def optimize_map_leg(dev, cfg, ba, calls=6, warm=2, iters=60):
    """Mapper.optimize_map (the reference entry point, Mapper.py:230-540) timed per call on the fused
    engine: `iters` joint iterations (middle 25 / fine 12 / colour 23 of 60), overlap keyframe selection
    over 4 keyframes (+ the last one and the current frame: a 5-frame window), frustum masks per call,
    a fresh Adam per call, BA of the 4 non-oldest cameras when `ba`.  Wall time of `calls` calls after
    `warm` (whose first captures the stage graphs), synchronised around."""
    P = pkg()
    scene = Room0Scene(dev, 0, cfg=dict(cfg), path="autograd")  # data only (grids, decoders, frames)
    for t in scene.grids.values():
        t.requires_grad_(False)
    mcfg = nice_slam_cfg(cfg)
    mp = P.Mapper(mcfg, None, slam_state(scene))
    mp.BA = ba
    F = cfg["window"]
    kf = [{"gt_c2w": _pose4(scene.c2w[f]), "idx": 50 * f, "depth": scene.depth[f], "color": scene.color[f],
           "est_c2w": _pose4(scene.c2w[f])} for f in range(F - 1)]
    kf_list = [50 * f for f in range(F - 1)]
    cur = _pose4(scene.c2w[F - 1])

    def call(k):
        return mp.optimize_map(iters, 1.0, 50 * F + 5 * k, scene.color[F - 1], scene.depth[F - 1], cur, kf, kf_list,
                               cur.clone())
    for k in range(warm):
        call(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(calls):
        call(warm + k)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / calls
    # where a call's time goes: extra calls with phase marks (host clock; HIP events on the stream)
    mp.timing = []
    for k in range(3):
        call(warm + calls + k)
    torch.cuda.synchronize()
    ph = ("masks", "selected", "window", "iterations")
    prev = ["t0"] + list(ph[:-1])
    host = {p: sum((t[p] - t[q]) * 1e3 for t in mp.timing) / len(mp.timing) for p, q in zip(ph, prev)}
    gpu = {p: sum(t["ev"][q].elapsed_time(t["ev"][p]) for t in mp.timing) / len(mp.timing)
           for p, q in zip(ph[1:], ph[:-1])}
    mp.timing = None
    res = {"ms_per_call": dt * 1e3, "ms_per_iteration": dt * 1e3 / iters, "iterations_per_call": iters,
           "calls": calls, "graphs_cached": len(mp._graphs), "bundle_adjustment": ba,
           "pixels": cfg["pixels"], "window": F,
           "phase_host_ms": {k: round(v, 3) for k, v in host.items()},
           "phase_gpu_ms": {k: round(v, 3) for k, v in gpu.items()},
           "iterations_gpu_ms_per_iteration": gpu["iterations"] / iters}
    del mp, scene
    torch.cuda.empty_cache()
    return res


def engine_stage_ms(dev, cfg, reps=50):
    """The bare engine (engine.MappingEngine.iteration, hipGraph blocks) per stage at a config's shape:
    what an optimize_map iteration of that stage costs without the drop-in's per-call work."""
    scene = Room0Scene(dev, 0, cfg=dict(cfg), path="fused")
    out = {}
    for stage in ("middle", "fine", "color"):
        out[stage], _ = graph_time(scene, lambda: scene.step(stage=stage), reps)
    out["schedule_60"] = (25 * out["middle"] + 12 * out["fine"] + 23 * out["color"]) / 60.0
    del scene
    torch.cuda.empty_cache()
    return {k: round(v, 4) for k, v in out.items()}


def engine_ba_stage_ms(dev, cfg, reps=50):
    """The bare engine with bundle adjustment per stage at a config's shape: engine.MappingEngine.iteration
    over the 5-frame window with d/dpts formed by the backward, the batched camera gradient of the 4
    non-oldest cameras (nslam_cam_grad_batch) and their Adam step, the poses re-derived from the cameras
    each iteration by the gather (nslam_frame.cam, ABI v21) — the GPU work of an optimize_map BA iteration, replayed in
    hipGraph blocks, without the drop-in's per-call work."""
    P = pkg()
    scene = Room0Scene(dev, 0, cfg=dict(cfg), path="fused")
    F = cfg["window"]
    n = cfg["pixels"] // F
    c2w = torch.eye(4, device=dev).repeat(F, 1, 1)
    c2w[:, :3] = scene.c2w
    cams = P.common.camera_tensors(c2w[1:]).contiguous()
    frames = [(scene.depth[0], scene.color[0], c2w[0])]
    frames += [(scene.depth[f], scene.color[f], c2w[f], cams[f - 1]) for f in range(1, F)]
    cgrad = torch.zeros_like(cams)
    ws = torch.zeros((F - 1) * P.ops.CAM_GRAD_WS_DOUBLES, dtype=torch.float64, device=dev)
    tk = torch.zeros(F - 1, dtype=torch.int32, device=dev)
    copt = P.ops.FusedAdam([{"params": [cams], "lr": 0.001}])
    eng = scene.engine

    def post_bwd(gps, ro, rd, z):
        P.ops.cam_grad_batch(cams, c2w[1:], [(1 + k) * n for k in range(F - 1)], n, gps, z, rd, cgrad, ws, tk)
        copt.step(grads={cams: cgrad})

    def step(stage):
        eng.iteration(stage, frames, None, n, (cfg["H"], cfg["W"]), (cfg["fx"], cfg["fy"], cfg["cx"], cfg["cy"]),
                      scene.opt, trainable_decoders=("color",), seed=1000, post_bwd=post_bwd)
    out = {}
    for stage in ("middle", "fine", "color"):
        out[stage], _ = graph_time(scene, lambda: step(stage), reps)
    out["schedule_60"] = (25 * out["middle"] + 12 * out["fine"] + 23 * out["color"]) / 60.0
    del scene
    torch.cuda.empty_cache()
    return {k: round(v, 4) for k, v in out.items()}


def slam_loop(dev, cfg=ROOM0, frames=60, warm_frames=10):
    """Measured room0 frames/s (BASELINE metric): the reference's per-frame work in one process on one
    stream — Tracker.track_frame every frame (10 camera iterations x 200 pixels, edges 100 px) and
    Mapper.optimize_map every 5th frame (60 iterations x 1000 pixels, 5-frame overlap window, frustum
    masks, BA of 4 cameras: the steady state after 4 keyframes, Mapper.run's every_frame / BA rule,
    Mapper.py:591-606), the tracker re-snapshotting the map after each mapping call (Tracker.py:130-142).
    Frames cycle through 5 synthetic keyframe views; the pose guess is the ground truth nudged by 2 cm.
    Wall time over `frames` frames after `warm_frames`, synchronised around."""
    P = pkg()
    scene = Room0Scene(dev, 0, cfg=dict(cfg), path="autograd")
    for t in scene.grids.values():
        t.requires_grad_(False)
    mcfg = nice_slam_cfg(cfg)
    slam = slam_state(scene)
    tr = P.Tracker(mcfg, None, slam)
    mp = P.Mapper(mcfg, None, slam)
    F = cfg["window"]
    kf = [{"gt_c2w": _pose4(scene.c2w[f]), "idx": 50 * f, "depth": scene.depth[f], "color": scene.color[f],
           "est_c2w": _pose4(scene.c2w[f])} for f in range(F)]
    kf_list = [50 * f for f in range(F)]
    nudge = torch.tensor([0.02, -0.01, 0.015], device=dev)
    stats = {"track_ms": [], "map_ms": []}

    def frame(i, timed_parts=False):
        f = i % F
        gt = _pose4(scene.c2w[f])
        pre = gt.clone()
        pre[:3, 3] += nudge
        t0 = time.perf_counter()
        est = tr.track_frame(i + 1, scene.color[f], scene.depth[f], gt, pre_c2w=pre)
        if timed_parts:
            torch.cuda.synchronize()
            stats["track_ms"].append((time.perf_counter() - t0) * 1e3)
        if i % 5 == 0:
            t0 = time.perf_counter()
            mp.BA = len(kf_list) > 4
            out = mp.optimize_map(60, 1.0, i + 1, scene.color[f], scene.depth[f], gt, kf, kf_list, est)
            slam.mapping_idx[0] = i + 1  # the tracker snapshots the new map before its next frame
            if timed_parts:
                torch.cuda.synchronize()
                stats["map_ms"].append((time.perf_counter() - t0) * 1e3)
            return out
        return est

    for i in range(warm_frames):
        frame(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(warm_frames, warm_frames + frames):
        frame(i)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for i in range(warm_frames + frames, warm_frames + frames + 10):  # component times (synchronised)
        frame(i, timed_parts=True)
    res = {"frames_per_s": frames / dt, "ms_per_frame": dt / frames * 1e3, "frames": frames,
           "track_frame_ms": sum(stats["track_ms"]) / len(stats["track_ms"]),
           "optimize_map_ms": sum(stats["map_ms"]) / max(len(stats["map_ms"]), 1),
           "tracker_graphs": len(tr._graphs), "mapper_graphs": len(mp._graphs),
           "workload": "room0 synthetic: track_frame every frame (10 x 200 px), optimize_map every 5th frame "
                       "(60 x 1000 px, window 5, frustum masks, BA), one process, one stream, measured wall time"}
    del tr, mp, scene
    torch.cuda.empty_cache()
    return res


def leg_main(leg):
    """One auxiliary measurement in this (child) process on cuda:0; prints one JSON object."""
    dev = torch.device("cuda", 0)
    if leg == "stress":
        res = stress_grid_query(dev)
    elif leg == "stress_iter":
        res = stress_iteration(dev)
    elif leg == "frame_io":
        res = frame_io(dev)
    elif leg == "apartment":
        res = apartment_iterations(dev)
    elif leg == "optimize_map":
        res = {"engine_ms_per_iteration": engine_stage_ms(dev, ROOM0),
               "engine_ba_ms_per_iteration": engine_ba_stage_ms(dev, ROOM0),
               "optimize_map": optimize_map_leg(dev, ROOM0, ba=False),
               "optimize_map_ba": optimize_map_leg(dev, ROOM0, ba=True)}
        for k, e in (("optimize_map", "engine_ms_per_iteration"), ("optimize_map_ba", "engine_ba_ms_per_iteration")):
            res[k]["vs_engine_schedule"] = res[k]["ms_per_iteration"] / res[e]["schedule_60"]
            res[k]["engine_baseline"] = e
        res["workload"] = ("Replica room0: Mapper.optimize_map(60 iterations, 1000 px over a 5-frame window) per call "
                           "vs the bare engine's iterations of the same stage mix (25 middle / 12 fine / 23 colour)")
    elif leg == "scene0000":
        res = {"engine_ms_per_iteration": engine_stage_ms(dev, SCENE0000),
               "engine_ba_ms_per_iteration": engine_ba_stage_ms(dev, SCENE0000),
               "optimize_map_ba": optimize_map_leg(dev, SCENE0000, ba=True)}
        om = res["optimize_map_ba"]
        om["vs_engine_schedule"] = om["ms_per_iteration"] / res["engine_ba_ms_per_iteration"]["schedule_60"]
        om["engine_baseline"] = "engine_ba_ms_per_iteration"
        om["ray_samples_per_s_upper"] = SCENE0000["pixels"] * 48 / (om["ms_per_iteration"] * 1e-3)
        res["workload"] = ("configs[2] ScanNet scene0000: 460x620, Mapper.optimize_map with BA over a 5-frame window "
                           "(4 cameras), 5000 px x 48 samples, 60 iterations per call")
    elif leg == "slam_loop":
        res = slam_loop(dev)
    else:
        scene = Room0Scene(dev, 0, cfg=dict(ROOM0), path="fused")
        for _ in range(3):
            scene.step()
        torch.cuda.synchronize()
        res = room0_frame_rate(scene) if leg == "frames" else bulk_queries(scene)
    print(json.dumps(res))


def run_leg(leg, timeout=300):
    """Spawn `bench.py --leg <leg>` as a child process (not an exec of this GPU process) and return
    its JSON, or an error record if it failed."""
    import subprocess
    try:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--leg", leg], capture_output=True, text=True,
                           timeout=timeout)
    except subprocess.TimeoutExpired:
        return {"error": f"leg {leg} timed out after {timeout} s"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        print(r.stderr[-2000:], file=sys.stderr)
        return {"error": f"leg {leg} exited with {r.returncode}"}
    return json.loads(lines[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--eager", action="store_true", help="no hipGraph capture")
    ap.add_argument("--serial-branches", action="store_true",
                    help="the backward's branches one after the other (counter passes: every kernel alone "
                         "on the chip, so its GRBM window holds no other work)")
    ap.add_argument("--no-stress", action="store_true", help="skip the 512^3 grid-query HBM measurement")
    ap.add_argument("--no-frames", action="store_true", help="skip the room0 frames/s (tracking + mapping stages)")
    ap.add_argument("--no-bulk", action="store_true", help="skip the forward-only mesher / render_img queries")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="process-group backend for N>1 (gloo: rehearse the sharded path on one GPU, eager)")
    ap.add_argument("--pixels", type=int, default=None,
                    help="override mapping pixels per iteration (scaling studies; the metric uses room0's 1000)")
    ap.add_argument("--path", choices=("fused", "autograd"), default="fused",
                    help="fused engine (default) or the autograd drop-in path")
    ap.add_argument("--exchange", choices=("sharded", "allreduce"), default="allreduce",
                    help="N>1 gradient exchange: all-reduce + replicated Adam (default) or sharded Adam")
    ap.add_argument("--force-exchange", action="store_true",
                    help="one rank: run the exchange's collectives anyway over a one-rank RCCL group "
                         "(identities), captured in the hipGraph like an N>1 job's")
    ap.add_argument("--no-prefetch", action="store_true",
                    help="draw + sample each iteration's rays inside it (no overlap with the previous backward)")
    ap.add_argument("--leg", choices=("frames", "stress", "stress_iter", "bulk", "frame_io", "apartment", "optimize_map",
                                      "scene0000", "slam_loop"), default=None,
                    help="run one auxiliary measurement and print its JSON (bench.py spawns these itself)")
    args = ap.parse_args()
    global PREFETCH, EXCHANGE, FORCE_EXCHANGE
    PREFETCH = not args.no_prefetch
    EXCHANGE = args.exchange
    FORCE_EXCHANGE = args.force_exchange
    if args.leg:
        return leg_main(args.leg)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.backend == "gloo":  # rehearsal of the sharded path with several ranks on one GPU
        local = local % max(torch.cuda.device_count(), 1)
    if args.force_exchange and world != 1:
        raise SystemExit("--force-exchange is the one-rank rehearsal of the exchange")
    if world > 1 or args.force_exchange:
        torch.cuda.set_device(local)
        if world == 1:  # not under torch.distributed.run: a one-rank rendezvous of our own
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local)
    P = pkg()
    cfg = dict(ROOM0)
    if args.pixels:
        cfg["pixels"] = args.pixels
    scene = Room0Scene(dev, rank, cfg=cfg, path=args.path)
    if args.serial_branches and getattr(scene, "engine", None) is not None:
        scene.engine.concurrent = False
    sharded = world > 1 or args.force_exchange
    for _ in range(args.warmup):
        scene.step(sharded=sharded)
    torch.cuda.synchronize()
    graph, mode = None, "eager"
    if not args.eager and not (world > 1 and args.backend == "gloo"):
        try:  # whole mapping iterations as hipGraphs (removes per-op host launch cost); two of them,
            # replayed in turn, since the prefetching engine alternates its ray buffers
            # blocks of GRAPH_BLOCK iterations per graph whatever --steps is (a replay starts only
            # after the previous one drained, ~20 us, paid once per block)
            graph, mode = capture_step_graphs(lambda: scene.step(sharded=sharded), sync=scene.flip_parity)
        except Exception as e:  # pragma: no cover - fall back to eager launches
            print(f"graph capture failed, eager mode: {e!r}", file=sys.stderr)
            graph, mode = None, "eager"
        if world > 1:
            # every rank replays graphs or every rank launches eagerly: a rank whose capture failed
            # would otherwise issue fewer collectives than the others and the job would hang
            ok = torch.tensor([0 if graph is None else 1], dtype=torch.int32, device=dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if int(ok.item()) == 0:
                graph, mode = None, "eager"
        if graph is not None:
            graph.run(graph.block)
            torch.cuda.synchronize()
    scene.kept.zero_()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if graph is not None:
        graph.run(args.steps)
    else:
        for _ in range(args.steps):
            scene.step(sharded=sharded)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    samples = int(scene.kept) * (cfg["n_strat"] + cfg["n_surf"])
    # per-kernel durations: HIP events around each C-ABI launch, on the launching stream, over
    # extra eager steps of the same kernels (events cannot bracket single kernels inside a replay)
    if graph is not None:
        graph.finish()
    timers = span_timers(scene, max(5, args.steps // 4), sharded=sharded)
    tot = torch.tensor([samples, dt], dtype=torch.float64, device=dev)
    if world > 1:
        s = tot[:1].clone()
        dist.all_reduce(s)
        m = tot[1:].clone()
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        samples_all, dt_max = float(s), float(m)
    else:
        samples_all, dt_max = float(samples), dt
    if rank == 0:
        pts_per_step = samples / args.steps
        qf = timers.get("query_fwd", {"avg_ms": float("nan")})
        qb = timers.get("query_bwd", {"avg_ms": float("nan")})
        # the dominant single launch (query_bwd is the span over its concurrent branches)
        dom_name, dom = max(((k, v) for k, v in timers.items() if k in KERNEL_WORK),
                            key=lambda kv: kv[1]["total_ms"])
        roof = kernel_roofline(dom_name, dom["avg_ms"], pts_per_step)
        per_kernel = {k: kernel_roofline(k, v["avg_ms"], pts_per_step) for k, v in timers.items() if k in KERNEL_WORK}
        out = {
            "metric": "ray-samples/sec (fwd+bwd) per mapping iter; frames/sec on Replica room0",
            "value": samples_all / dt_max, "unit": "ray-samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt_max / args.steps * 1e3, "higher_is_better": True,
            "launch_mode": mode, "ray_prefetch": PREFETCH,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32 (z, depth, var in f64)",
            "data": "synthetic room0-shaped frames (analytic depth, random colour), seeded random-init decoders",
            "config": {"workload": "Replica room0 mapping iteration, colour stage: 1000 pixels x 48 samples "
                                   "(5-frame window x 200), grids middle/fine/colour, Adam",
                       "global_batch": int(round(pts_per_step)) * world, "seq_len": 48,
                       "parallelism": f"rays sharded dp{world}, RCCL all-reduce of the frustum-row gradients"},
            "roofline": roof,
            "kernel_rooflines": per_kernel,
            "kernels_ms": {k: round(v["avg_ms"], 4) for k, v in timers.items()},
            "query_fwd_hbm_frac": (pts_per_step * BYTES_FWD_PER_SAMPLE / (qf["avg_ms"] * 1e-3) / 1e9) / HBM_PEAK_GBS
            if "query_fwd" in timers else None,
            "graph_block": GRAPH_BLOCK,
            "query_bwd_ms": qb["avg_ms"],
        }
        if sharded and args.path == "fused":
            keys, dn = scene.engine.grads_for("color", ("color",))
            out["exchange_bytes_per_step"] = scene.exchange.payload_bytes(keys, dn)
            out["exchange"] = EXCHANGE
            out["exchange_backend"] = dist.get_backend() if dist.is_initialized() else None
            out["exchange_forced_world1"] = bool(args.force_exchange)
            # the collectives' own HIP-event spans (eager iterations, branches serialised), per iteration
            coll = {k: v for k, v in timers.items() if k.startswith("collective.")}
            out["collective_ms_per_step"] = {k: round(v["total_ms"] / max(5, args.steps // 4), 4)
                                             for k, v in coll.items()}
            out["dense_grad_bytes_per_step"] = sum(v.numel() for v in scene.grids.values()) * 4
        # the auxiliary measurements run as child processes: a failure there (one run on a fresh
        # box ended in a host heap abort inside a later leg) cannot take the headline line with it
        if world == 1 and not args.no_frames and args.path == "fused":
            out["room0"] = run_leg("frames")
            out["room0_slam_loop"] = run_leg("slam_loop")
            out["optimize_map"] = run_leg("optimize_map")
            out["scene0000_ba"] = run_leg("scene0000")
            out["apartment"] = run_leg("apartment")
        if world == 1 and not args.no_stress:
            out["grid_query_stress"] = run_leg("stress")
            out["stress_iteration"] = run_leg("stress_iter")
        if world == 1 and not args.no_bulk:
            out["bulk_forward"] = run_leg("bulk")
            out["frame_io"] = run_leg("frame_io")
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(scene)
            ref = reference_gpu_baseline(scene)
            out["reference_gpu_path"] = ref
            out["vs_reference_gpu_path"] = out["value"] / ref["value"]
        print(json.dumps(out))
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
