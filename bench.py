"""bench.py -- train views/sec (fwd+bwd raster) @1080p, 1e6 Gaussians; 1/2/4/8-GPU ADMM scaling.

One step = one view per rank: _C.rasterize_gaussians + _C.rasterize_gaussians_backward on the synthetic 1080p scene of
BASELINE.md §2 / SURVEY.md §8(d) (SH degree 3, AA off, fixed random dL/dcolor, zero dL/dinvdepth), inputs resident in
HBM.  The steps cycle through --views seeded yaw views (camera at the origin rotated about +y, yaw ~ U[-10, 10] deg
from seed 1234, view 0 = yaw 0; SURVEY.md §8(d) "vary the camera yaw to build view batches").  With N > 1 ranks
(torch.distributed.run, one GPU each, RCCL) every rank renders its own scene block and the ADMM consensus all_reduce
of the shared Gaussians is added in its 1-per-200-iterations proportion.  value = views of all ranks / max-over-ranks
time.

Also reported on the same JSON line:
  views         per view: yaw, num_rendered, the reference's precise instance count K (its full per-tile lists, one
                untimed forward with depth-prefix binning off), this build's binned instances (phase 1 E1 + phase 2
                E2), visible / binned / gradient-carrying Gaussians
  roofline      the dominant kernel (most time per view, hipEvent-timed on the launch stream over one extra pass of
                the views) credited with the algorithmic bytes of the work it performs (phase_bytes: binned
                instances, not the reference's K); the view total over the same model (view_frac); the reference-
                equivalent figure of SURVEY.md §8(d) (B_view = 856 N + 172 K + 64 HW, the reference's work) kept
                apart; HBM `traffic` and a VALU-issue roofline of the render kernels from the committed rocprofv3 PMC
                passes of the same command (profiles/pmc_traffic.json), when present
  cpu_baseline  the CPU oracle (oracle/gs_oracle.c, the reference kernels restated; OpenMP, results identical for
                any thread count) on the same views: all host threads of this job, and one core
  train_step    secondary figure: activations + fwd + L1 + fused-SSIM fwd/bwd + bwd + densification statistics +
                SparseGaussianAdam (6 groups, one launch) over the same views, and one densify_and_prune
  admm          N > 1 (or --admm): the ADMM block trainer (dogs_amd.admm_trainer) run for --admm-iters local
                iterations per rank with a consensus every --admm-interval, and its sequential single-GPU equivalent
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "train views/sec (fwd+bwd raster) @1080p, 1e6 Gaussians; 1/2/4/8-GPU ADMM scaling"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
SIMDS, CLOCK_GHZ = 1024, 2.4   # 256 CUs x 4 SIMDs; a wave64 VALU instruction issues over 2 cycles (SIMD-32)
VALU_PEAK_GINST = SIMDS * CLOCK_GHZ / 2.0   # 1228.8 G wave-instructions/s


def phase_bytes(phase: str, v: dict) -> float:
    """Algorithmic bytes of the work each phase performs on one view (DESIGN.md §3 "Roofline"):
    N Gaussians, Vis visible (radii > 0), Gb binned (>= 1 instance), Gl gradient-carrying, E1/E2 phase-1/phase-2
    instances (E = E1 + E2), HW pixels.  Per unit: preprocess reads means/scales/rotation/opacity (44 B) and writes the
    32-B splat record, depth key, rect count, instance count and radius (48 B); the depth histogram reads key + count;
    the binning walk reads the splat record twice (count, emit) and, for the SH colour, means + dc + rest (204 B) and
    writes rgb/inv-depth (16 B) per binned Gaussian, and writes Gaussian, depth key and tile slot (12 B) per instance;
    the render gathers 44 B per instance (id, xy, conic/opacity, rgb, depth) and its fused sort reads key + id and
    writes the sorted id (12 B), and writes colour, inverse depth, T and last contributor (24 B/px); the replay
    re-gathers 44 B and writes one 40-B record per instance and reads 40 B/px, and its waves issue the zero fill of the
    dense gradient outputs (288 B per Gaussian, in the shadow of its VALU work: credited to the kernel that issues
    it); the per-Gaussian backward reads the records (40 B/instance) and 236 B of parameters + radius + 40-B sums per
    gradient-carrying Gaussian, and overwrites those Gaussians' output rows (counted in the fill)."""
    N, HW = v["N"], v["HW"]
    E1, E2 = v["e1"], v["e2"]
    E = E1 + E2
    Gb, Gl = v["binned_gaussians"], v["live_gaussians"]
    return {
        "preprocess": 92.0 * N,
        "prefix_cut": 8.0 * N,
        "emit": (64.0 + 220.0) * Gb + 12.0 * E1,
        "tile_bin": 0.0,
        "render_fwd": 56.0 * E1 + 24.0 * HW,
        "phase2": 68.0 * E2,
        "render_bwd": 84.0 * E + 40.0 * HW + 288.0 * N,
        "gauss_bwd": 40.0 * E + 280.0 * Gl,
    }.get(phase, 0.0)


def reference_view_bytes(N: int, K: int, HW: int) -> float:
    """the reference's algorithmic bytes per view (its full lists, K precise instances)."""
    return 856.0 * N + 172.0 * K + 64.0 * HW


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return int(sk.getsockname()[1])


def relaunch_command(gpus: int | None, argv: list, environ) -> list | None:
    """`bench.py --gpus N` (N > 1) outside a launcher: the torch.distributed.run command that runs it as N ranks, one
    per GPU (the reference launches its trainer the same way, scripts/train/train_admm_master.sh:34-42); None when
    this process is already a rank or N <= 1."""
    if gpus is None or gpus <= 1 or "WORLD_SIZE" in environ:
        return None
    argv = ["--gaussians" if a == "--n" else ("--gaussians=" + a[4:] if a.startswith("--n=") else a) for a in argv]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__), *argv]


def check_world(gpus: int | None, ws: int) -> None:
    if gpus is not None and gpus != ws:
        raise SystemExit(f"bench.py: --gpus {gpus} but the launcher started {ws} rank(s) (WORLD_SIZE)")


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def view_yaws(views: int, seed: int = 1234):
    """Seeded yaw batch (degrees): view 0 looks down +z, the others yaw ~ U[-10, 10]."""
    return [0.0] + [float(x) for x in np.random.default_rng(seed).uniform(-10.0, 10.0, max(views - 1, 0))]


def make_cameras(W, H, yaws, dev, fx=1600.0):
    import math
    from dogs_amd.camera import make_camera, yaw_world_to_camera
    return [make_camera(W, H, fx, fx, world_to_camera=yaw_world_to_camera(math.radians(y))).to(dev) for y in yaws]


class Views:
    """One fwd+bwd raster step per call through the drop-in `_C` table, cycling through the view cameras."""

    def __init__(self, s, cams, grad_color, grad_inv, dev):
        from dogs_amd.diff_gaussian_rasterization import _C
        self._C = _C
        self.s, self.cams, self.gc, self.gi, self.dev = s, cams, grad_color, grad_inv, dev
        self.bg = torch.zeros(3, device=dev)
        self.e = torch.empty(0, device=dev)
        self.i = 0

    def forward(self, c):
        s, e = self.s, self.e
        return self._C.rasterize_gaussians(self.bg, s.means3D, e, s.opacities, s.scales, s.rotations, 1.0, e,
                                           c.world_to_camera, c.projective_matrix, c.tanfovx, c.tanfovy, c.height,
                                           c.width, s.dc, s.sh, 3, c.camera_center, False, False, False)

    def backward(self, c, out):
        s, e = self.s, self.e
        return self._C.rasterize_gaussians_backward(self.bg, s.means3D, out[4], e, s.opacities, s.scales, s.rotations,
                                                    1.0, e, c.world_to_camera, c.projective_matrix, c.tanfovx,
                                                    c.tanfovy, self.gc, s.dc, s.sh, self.gi, 3, c.camera_center,
                                                    out[5], out[0], out[6], out[7], out[1], out[8], False, False)

    def step(self):
        c = self.cams[self.i % len(self.cams)]
        self.i += 1
        out = self.forward(c)
        return out, self.backward(c, out)

    def stats(self, k, reference_k=True):
        """Untimed per-view figures: counters of a normal forward, the gradient-carrying Gaussians of its backward,
        and the reference's precise instance count K (one forward with depth-prefix binning off)."""
        import dogs_amd._lib as L
        c = self.cams[k]
        out = self.forward(c)
        g = self.backward(c, out)
        n = int(self.s.means3D.shape[0])
        cnt = L.forward_counters(out[5], n)
        tile_count = torch.empty(n, dtype=torch.int32, device=self.dev)
        L.check(L.load().dg_debug_geometry(out[5].data_ptr(), n, None, None, None, tile_count.data_ptr(),
                                           L.stream_of(self.dev)))
        rec = {"num_rendered": int(out[0]), "e1": cnt["e1"], "e2": cnt["e2"],
               "unfinished_tiles": cnt["unfinished_tiles"] if cnt["cut"] else 0,
               "visible_gaussians": int((out[4] > 0).sum()), "binned_gaussians": int((tile_count > 0).sum()),
               "live_gaussians": int((g[2].reshape(-1) != 0).sum())}
        if not reference_k:
            rec["K"] = -1
            return rec
        old = self._C.set_prefix_per_tile(-1)
        try:
            ref = self.forward(c)
            rec["K"] = L.forward_counters(ref[5], n)["e1"]
        finally:
            self._C.set_prefix_per_tile(old)
        return rec


class TrainStep:
    """Training iteration of GaussianSplatTrainer.train_iteration (gaussian_trainer.py:324-513) before
    densify_end_iter, without the periodic densify_and_prune: activations, raster, L1 + fused-SSIM, backward, the
    view's densification statistics (:433-438) and SparseGaussianAdam.step(visible, N) -- the last two in one
    launch -- cycling through the view cameras.  densify() times one densify_and_prune (dogs_amd.densify)."""

    def __init__(self, s, cams, dev, seed):
        from dogs_amd.diff_gaussian_rasterization import (GaussianRasterizationSettings, GaussianRasterizer,
                                                          SparseGaussianAdam)
        from dogs_amd.activations import activate
        from dogs_amd.fused_ssim import fused_ssim
        from dogs_amd.loss import clamp_l1, row_prod
        self.activate, self.clamp_l1, self.fused_ssim = activate, clamp_l1, fused_ssim
        self.row_prod = row_prod  # prod(dim=1) without prod_backward's host read of the zero count
        self.cams = cams
        self.rasts = [GaussianRasterizer(GaussianRasterizationSettings(
            c.height, c.width, c.tanfovx, c.tanfovy, torch.zeros(3, device=dev), 1.0, c.world_to_camera,
            c.projective_matrix, 3, c.camera_center, False, False, False, 0.0)) for c in cams]
        self.i = 0
        self.params = {
            "xyz": s.means3D.clone().requires_grad_(True),
            "f_dc": s.dc.clone().requires_grad_(True),
            "f_rest": s.sh.clone().requires_grad_(True),
            "scaling": s.raw_scales.to(dev).clone().requires_grad_(True),
            "quaternion": s.raw_rotations.to(dev).clone().requires_grad_(True),
            "opacity": s.raw_opacities.to(dev).clone().requires_grad_(True),
        }
        lrs = {"xyz": 1.6e-4, "f_dc": 2.5e-3, "f_rest": 1.25e-4, "scaling": 5e-3, "quaternion": 1e-3, "opacity": 2.5e-2}
        self.opt = SparseGaussianAdam([{"params": [p], "lr": lrs[k], "name": k} for k, p in self.params.items()],
                                      lr=0.0, eps=1e-15)
        c = cams[0]
        g = torch.Generator().manual_seed(seed + 7)
        self.gt = torch.rand((3, c.height, c.width), generator=g).to(dev)
        N = s.means3D.shape[0]
        self.stats = {"max_radii2D": torch.zeros(N, device=dev), "grad_accum": torch.zeros((N, 1), device=dev),
                      "denom": torch.zeros((N, 1), device=dev)}

    def step(self):
        p = self.params
        rast = self.rasts[self.i % len(self.rasts)]
        self.i += 1
        m2d = torch.zeros_like(p["xyz"], requires_grad=True)
        # get_opacity / get_scaling / get_quaternion (sigmoid, exp, normalize) fused in one launch each way
        opac, scales, rots = self.activate(p["opacity"], p["scaling"], p["quaternion"])
        img, radii, _ = rast(means3D=p["xyz"], means2D=m2d, opacities=opac, dc=p["f_dc"], shs=p["f_rest"],
                             scales=scales, rotations=rots)
        img, l1 = self.clamp_l1(img, self.gt)  # render()'s clamp + the L1 term, one launch each way
        ssim = self.fused_ssim(img.unsqueeze(0), self.gt.unsqueeze(0))
        # gaussian_trainer.py:387-408: lambda_dssim 0.2, lambda_scale 0.05 (urban3d_admm.yaml loss block)
        loss = 0.8 * l1 + 0.2 * (1.0 - ssim) + 0.05 * self.row_prod(scales).mean()
        loss.backward()
        vis = radii > 0
        self.opt.step(vis, radii.shape[0], stats=dict(self.stats, radii=radii, dmeans2D=m2d.grad))
        self.opt.zero_grad(set_to_none=True)

    def native(self):
        """The same iteration through dg_train_step (dogs_amd.train_step): one C call per view."""
        from dogs_amd.train_step import NativeTrainStep
        p = self.params
        params = {"xyz": p["xyz"], "features_dc": p["f_dc"], "features_rest": p["f_rest"], "opacity": p["opacity"],
                  "scaling": p["scaling"], "quaternion": p["quaternion"]}
        # overlap: each step's f_dc / f_rest update runs beside the next step's forward up to its emission (the
        # timed region's closing torch.cuda.synchronize() waits for it like for everything else)
        nts = NativeTrainStep(params, self.opt, self.cams, [self.gt] * len(self.cams), 3, 0.2, 0.05,
                              torch.zeros(3, device=self.gt.device), self.gt.device, stats=self.stats, overlap=True)
        state = {"i": 0}

        def step():
            nts.step(state["i"] % len(self.cams))
            state["i"] += 1
        return step

    def densify(self):
        """One densify_and_prune (urban3d.yaml thresholds: grad 2e-4, percent_dense 0.01, min opacity 0.005,
        max_screen_size 20) on the current state: wall ms including its two host syncs."""
        import types
        from dogs_amd import densify
        p = self.params
        model = types.SimpleNamespace(percent_dense=0.01, xyz_gradient_accum=self.stats["grad_accum"],
                                      denom=self.stats["denom"], max_radii2D=self.stats["max_radii2D"])
        for k, a in zip(densify.NAMES, densify.ATTRS):
            setattr(model, a, p[k])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n_out = densify.densify_and_prune(model, 2e-4, 0.005, 5.0, 20.0, self.opt)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3, n_out


def masked_iteration_leg(s, cams, dev, seed, iters=40, warmup=10) -> dict:
    """BASELINE config 2's iteration as the trainer runs it: GaussianSplatTrainer (native route) with
    mipnerf360.yaml's options -- the appearance mask (geometry.mask, lambda_mask 0), lambda_dssim 0.2, lambda_scale
    0.01, SH degree 3, densification statistics on -- on the bench scene and views; densify / reset events moved past
    the timed window (their cost is one densify_and_prune per 100 iterations, reported apart in train_step).  The yaml's
    values come from the committed parse of the reference file (tests/golden/reference_configs.json)."""
    from dataclasses import replace
    from dogs_amd.gaussian_model import GaussianSplatModel
    from dogs_amd.trainer import GaussianSplatTrainer, GSTrainConfig
    with open(os.path.join(ROOT, "tests", "golden", "reference_configs.json")) as f:
        cfg = GSTrainConfig.from_reference(json.load(f)["mipnerf360.yaml"])
    cfg = replace(cfg, densify_start_iter=10 ** 9, opacity_reset_interval=10 ** 9, spatial_lr_scale=1.0)
    m = GaussianSplatModel(3, cfg.percent_dense, dev)
    m.init_from_external_properties(s.means3D, s.dc, s.sh, s.raw_scales, s.raw_rotations, s.raw_opacities)
    m.active_sh_degree = 3
    g = torch.Generator().manual_seed(seed + 11)
    gts = [torch.rand((3, c.height, c.width), generator=g).to(dev) for c in cams]
    torch.manual_seed(seed)
    tr = GaussianSplatTrainer(m, cams, gts, cfg, device=dev, seed=seed, native=True)
    for _ in range(warmup):
        tr.train_iteration()
    tr.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        tr.train_iteration()
    tr.sync()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / iters * 1e3
    out = {"ms_per_iteration": round(ms, 3), "iterations_per_s": round(1e3 / ms, 1), "iterations": iters,
           "includes": "appearance-embedding forward (dg_conv3x3 + dg_mask_head_forward) + dg_train_step (raster "
                       "fwd/bwd, masked L1, fused SSIM, scale regulariser, statistics, SparseGaussianAdam) + the "
                       "embedding's backward (dg_mask_head_backward, dg_conv3x3 adjoint, dg_conv3x3_wgrad) and Adam",
           "config": "mipnerf360.yaml (geometry.mask true, lambda_mask 0, lambda_dssim 0.2, lambda_scale 0.01), "
                     "1e6 Gaussians at 1920x1080, native route"}
    del tr, m, gts
    torch.cuda.empty_cache()
    return out


def host_threads() -> int:
    """Threads this job may use on the host: OMP_NUM_THREADS when the launcher sets it (the GPU box grants a share of
    a bigger machine), else the CPUs this process may run on."""
    try:
        n = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        n = 0
    if n > 0:
        return n
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline(n, W, H, seed, yaws, budget_s=12.0):
    """The CPU oracle (the reference's kernels restated in C; the reference has no CPU rasterizer) on
    the same views, fwd+bwd: all host threads of this job, then one core.  Each leg runs whole views in the bench's
    view order until its time budget is spent (at least one view)."""
    from oracle import oracle as O
    from dogs_amd.synthetic import make_scene
    O.build()
    s = make_scene(n, W, H, seed=seed)
    cams = make_cameras(W, H, yaws, torch.device("cpu"))
    g = torch.Generator().manual_seed(seed + 99)
    gc = torch.randn((3, H, W), generator=g).numpy()
    prm = dict(dc=s.dc.numpy(), sh=s.sh.numpy(), scales=s.scales.numpy(), rotations=s.rotations.numpy())
    means, opac = s.means3D.numpy(), s.opacities.numpy()

    def leg(threads):
        old = O.set_threads(threads)
        try:
            done, t0 = 0, time.perf_counter()
            while True:
                c = cams[done % len(cams)]
                _, _, _, st = O.forward(means, opac, c.world_to_camera.numpy(), c.projective_matrix.numpy(),
                                        c.camera_center.numpy(), c.tanfovx, c.tanfovy, H, W, np.zeros(3, np.float32),
                                        **prm)
                st.backward(gc)
                del st
                done += 1
                dt = time.perf_counter() - t0
                if dt >= budget_s or done >= 4 * len(cams):
                    return done, dt, O.get_threads()
        finally:
            O.set_threads(old)

    threads = host_threads()
    nv_all, dt_all, used = leg(threads)
    nv_one, dt_one, _ = leg(1)
    try:
        model = [l for l in open("/proc/cpuinfo") if l.startswith("model name")][0].split(":", 1)[1].strip()
    except Exception:  # noqa: BLE001
        model = "unknown"
    return {"value": round(nv_all / dt_all, 4), "unit": "views/s", "cores": used, "kind": "port",
            "sample": f"{nv_all} views fwd+bwd of the same {W}x{H} / {n}-Gaussian yaw batch, {used} OpenMP threads "
                      f"({model}; os.cpu_count()={os.cpu_count()})",
            "seconds": round(dt_all, 3),
            "single_core": {"value": round(nv_one / dt_one, 4), "unit": "views/s", "cores": 1,
                            "sample": f"{nv_one} views, 1 thread", "seconds": round(dt_one, 3)}}


def _grid(blocks: int) -> tuple:
    """mx x my of the Grid2D split for a block count (one block per rank)."""
    mx = 1
    while mx * mx < blocks:
        mx *= 2
    return mx, max(1, blocks // mx)


def admm_leg(args, ws, rank, dev, n, W, H):
    """The ADMM trainer end to end (dogs_amd.admm_run, master_gaussian_trainer.py:620-728): a synthetic aerial scene of
    ~n points per block split by the Grid2D path into one block per rank (2 x 1, 2 x 2, 4 x 2), nadir cameras at W x H
    with seeded smooth targets; every rank runs `run()`: --admm-pre pre-phase iterations with densification (the
    GaussianSplatTrainer loop: native steps, densify / reset on the autograd route), the phase entry (all-gather + fuse,
    count renders of its own cameras, the order-exact importance fold, prune, expanded-box split), then --admm-rounds
    rounds of --admm-interval local steps (activations, raster fwd/bwd, L1 + SSIM + scale regulariser, SparseGaussianAdam
    with the ADMM penalty) + consensus (RCCL all_reduce of the shared Gaussians, duals, residuals, rho adaptation).
    Rank 0 then runs the same split block after block on its one GPU (`run_sequential`, the single-GPU baseline of the
    '>= 6x at 8 GPUs' target): speedup = sequential / parallel wall time, for the whole run and for the ADMM rounds.
    At one rank the split has 2 blocks and only the sequential run is timed."""
    import gc
    import tempfile
    from dogs_amd.admm import ADMMConfig
    from dogs_amd.admm_run import ADMMRunConfig, aerial_views, run, run_sequential, split_scene
    from dogs_amd.trainer import GSTrainConfig
    nb = ws if ws > 1 else 2
    mx, my = _grid(nb)
    pre = max(0, args.admm_pre)
    rounds = max(1, args.admm_rounds)
    gs = GSTrainConfig(max_iterations=pre + rounds * args.admm_interval, densify_start_iter=min(50, pre // 2),
                       densify_end_iter=pre, densification_interval=max(pre // 2, 1), opacity_reset_interval=10 ** 6,
                       prune_iterations=(), spatial_lr_scale=-1, percent_dense=0.001, lambda_scale=0.05,
                       position_init=0.000016, position_final=0.00000016, position_max_iterations=30000, opacity=0.05)
    cfg = ADMMRunConfig(gs=gs, admm=ADMMConfig(consensus_interval=args.admm_interval))
    with tempfile.TemporaryDirectory() as tmp:
        # n * nb / 2 points on a (8 mx) x (8 my) slab: each block's expanded cell (1.4 x 1.4 of its cell) holds about n
        # of them; 2 x 2 nadir cameras per cell, 4 apart, at height 6: footprints 8.4 x 4.7, so every point is seen
        # and the overlaps hold shared Gaussians after the entry's importance prune
        views = aerial_views(n * nb // 2, 2 * mx, 2 * my, W, H, extent=(4.0 * mx, 4.0 * my), height=6.0, seed=77)
        scenes = split_scene(views, mx, my, tmp, dev, image_seed=78)
        # untimed warm-up on the same split (allocator, adaptive capacity, first-call library setup), so that neither
        # the parallel nor the sequential timing carries one-time costs
        warm = ADMMRunConfig(gs=GSTrainConfig(**{**gs.__dict__, "max_iterations": 40, "densify_end_iter": 20,
                                                 "densify_start_iter": 5, "densification_interval": 10}),
                             admm=ADMMConfig(consensus_interval=20))
    out = {"blocks": nb, "grid": [mx, my], "pre_phase_iterations": pre, "rounds": rounds,
           "interval": args.admm_interval, "points_per_block": [int(sc.points.shape[0]) for sc in scenes],
           "cameras_per_block": [len(c) for c in scenes[0].camera_blocks],
           "includes": "pre-phase (densify) + phase entry (fuse, count renders, importance prune, re-split) + ADMM "
                       "rounds (local steps: activations + raster fwd/bwd + clamp/L1 + fused SSIM + scale regulariser "
                       "+ SparseGaussianAdam with the proximal gradient; consensus all_reduce of the shared set, "
                       "duals, residuals, rho adaptation)"}
    if ws > 1:
        run(warm, scenes[rank], device=dev, seed=5)
    else:
        run_sequential(warm, scenes, dev, seed=5)
    gc.collect()
    torch.cuda.empty_cache()
    if ws > 1:
        from dogs_amd.admm_trainer import barrier_time
        res = {}
        t_par = barrier_time(lambda: res.update(r=run(cfg, scenes[rank], device=dev, seed=5)), dev, ws)
        r = res["r"]
        secs = {k: max_over(ws, dev, v) for k, v in r.seconds.items()}
        steps = rounds * args.admm_interval
        out.update({"seconds": round(t_par, 3), "phase_seconds": {k: round(v, 3) for k, v in secs.items()},
                    "views_per_s": round(ws * steps / secs["admm"], 2),
                    "gaussians_per_block_admm": int(r.block.params["xyz"].shape[0]),
                    **({"entry_stages_s": {k: round(max_over(ws, dev, v), 4) for k, v in r.entry.timings.items()}}
                       if r.entry.timings else {}),
                    "num_global": r.entry.num_global, "shared_gaussians": r.consensus.num_shared,
                    "consensus_ms": round(1e3 * max(lg.seconds["consensus"] for lg in r.runner.logs), 3),
                    "last_round": {"primal": {k: float(f"{v:.4g}") for k, v in r.runner.logs[-1].primal.items()},
                                   "dual": {k: float(f"{v:.4g}") for k, v in r.runner.logs[-1].dual.items()}}})
        # rank 0's block at the end, for the bit-for-bit comparison with the sequential baseline below
        mine = [t.detach().clone() for t in r.block.param_tuple()] if rank == 0 else None
        del res, r
        gc.collect()
        torch.cuda.empty_cache()
        dist.barrier()
    if rank == 0:
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        seq = run_sequential(cfg, scenes, dev, seed=5)
        torch.cuda.synchronize(dev)
        t_seq = time.perf_counter() - t0
        if ws > 1:   # the same trajectory: every parameter of block 0 bit for bit (the consensus and capacity contexts)
            out["rank0_equals_sequential"] = bool(all(torch.equal(a, b.detach())
                                                      for a, b in zip(mine, seq.blocks[0].param_tuple())))
            del mine
        out["sequential"] = {"blocks": nb, "seconds": round(t_seq, 3),
                             "phase_seconds": {k: round(v, 3) for k, v in seq.seconds.items()},
                             "views_per_s": round(nb * rounds * args.admm_interval / seq.seconds["admm"], 2),
                             "shared_gaussians": seq.seq.cons.num_shared, "num_global": seq.entries[0].num_global}
        if ws > 1:
            out["speedup_vs_sequential"] = round(t_seq / out["seconds"], 3)
            out["speedup_admm_rounds"] = round(seq.seconds["admm"] / out["phase_seconds"]["admm"], 3)
        del seq
        gc.collect()
        torch.cuda.empty_cache()
    if ws > 1:
        dist.barrier()
    return out


SWEEP = (  # (name, N, W, H, raw-opacity mean): north_star's other N, the 4K config, and a non-saturating scene
    ("1e5@1080p", 100_000, 1920, 1080, 0.0),
    ("5e6@1080p", 5_000_000, 1920, 1080, 0.0),
    ("1e6@4K", 1_000_000, 3840, 2160, 0.0),
    ("1e6@1080p-sparse", 1_000_000, 1920, 1080, -2.0),
)


def phase_profile(views, yaws, vstats, pmc: dict) -> dict:
    """One profiled pass over the views (per-phase hipEvent durations on the stream the kernels run on): per phase
    its ms per view, the algorithmic bytes of the work it did (phase_bytes) and their fraction of the HBM peak, the
    dominant phase (the most time among phases with bytes), and the render kernels' VALU issue fraction when the PMC
    passes of this workload are committed (profiles/pmc_traffic.json)."""
    import dogs_amd._lib as L
    torch.cuda.synchronize()
    views.i = 0
    L.profile_enable(True)
    for _ in range(len(yaws)):
        views.step()
    torch.cuda.synchronize()
    prof = L.profile_collect()
    L.profile_enable(False)
    nv = float(len(yaws))
    phase_ms = {k: v[0] / nv for k, v in prof.items()}
    phase_b = {k: float(np.mean([phase_bytes(k, r) for r in vstats])) for k in phase_ms}
    dom = max(phase_ms, key=lambda k: phase_ms[k] if phase_b.get(k, 0) > 0 else -1.0)

    def valu(phase):
        e = pmc.get(phase)
        if not isinstance(e, dict) or "valu_insts" not in e:
            return None
        t = phase_ms[phase] * 1e-3
        out = {"insts": e["valu_insts"], "achieved_ginst_s": round(e["valu_insts"] / t / 1e9, 1),
               "peak_ginst_s": VALU_PEAK_GINST, "frac": round(e["valu_insts"] / t / 1e9 / VALU_PEAK_GINST, 4)}
        if "valu_busy" in e:
            out["busy"] = e["valu_busy"]
        if "hbm_bytes" in e:
            out["traffic"] = e["hbm_bytes"]
        return out

    return {"phase_ms_raw": phase_ms, "phase_b_raw": phase_b, "dominant": dom,
            "phases_ms": {k: round(v, 4) for k, v in sorted(phase_ms.items(), key=lambda kv: -kv[1])},
            "phase_bytes": {k: round(v) for k, v in phase_b.items() if v > 0},
            "phase_hbm_frac": {k: round(phase_b[k] / (phase_ms[k] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                               for k in phase_ms if phase_b.get(k, 0) > 0 and phase_ms[k] > 0},
            "view_bytes": float(sum(phase_b.values())),
            "valu": {k: valu(k) for k in ("render_bwd", "render_fwd") if k in phase_ms}}


def sweep_leg(dev, yaws, seed, steps=16, warmup=8, only=None):
    """After the headline: the same fwd+bwd view step (same yaw batch, cold adaptive capacity, warm-up, barrier-free
    single-rank timing) on the other workloads of SURVEY.md §8(d) / north_star -- N in {1e5, 5e6} at 1080p, 1e6 at
    3840x2160 -- and on a non-saturating variant of the 1080p / 1e6 scene (raw opacity ~ N(-2, 1.5): far fewer tiles
    saturate before their lists end, so most of the work is phase 2 and the depth prefix saves little).  Per entry:
    views/s, ms/view, mean E1 / E2 / unfinished tiles / K (the reference's precise instances) and the reference-
    equivalent view fraction (856 N + 172 K + 64 HW per view over 8 TB/s)."""
    import gc
    import dogs_amd._lib as L
    from dogs_amd.synthetic import make_scene
    out = {}
    for name, n, W, H, om in SWEEP:
        if only is not None and name not in only:
            continue
        s = make_scene(n, W, H, seed=seed, opacity_mean=om).to(dev)
        cams = make_cameras(W, H, yaws, dev)
        g = torch.Generator().manual_seed(seed + 99)
        v = Views(s, cams, torch.randn((3, H, W), generator=g).to(dev), torch.zeros((1, H, W), device=dev), dev)
        with torch.cuda.device(dev):
            L.adaptive_capacity(W, H, reset=True)
        for _ in range(warmup):
            v.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            v.step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        st = [v.stats(k) for k in range(len(yaws))]
        for r in st:
            r.update(N=n, HW=W * H)
        K = float(np.mean([r["K"] for r in st]))
        ref_b = reference_view_bytes(n, int(K), W * H)
        pmc_key = f"{n}x{W}x{H}" + ("-sparse" if om != 0.0 else "")
        prof = phase_profile(v, yaws, st, load_pmc_key(pmc_key))
        out[name] = {"N": n, "width": W, "height": H, "raw_opacity_mean": om,
                     "views_per_s": round(1e3 / ms, 2), "ms_per_view": round(ms, 4),
                     "e1_mean": round(float(np.mean([r["e1"] for r in st]))),
                     "e2_mean": round(float(np.mean([r["e2"] for r in st]))),
                     "unfinished_tiles_mean": round(float(np.mean([r["unfinished_tiles"] for r in st])), 1),
                     "K_mean": round(K), "tiles": ((W + 15) // 16) * ((H + 15) // 16),
                     "reference_equivalent_view_frac": round(ref_b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "view_frac": round(prof["view_bytes"] / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "dominant": prof["dominant"], "phases_ms": prof["phases_ms"],
                     "phase_bytes": prof["phase_bytes"], "phase_hbm_frac": prof["phase_hbm_frac"],
                     "valu": prof["valu"], "pmc_key": pmc_key}
        del v, s, cams, st
        gc.collect()
        torch.cuda.empty_cache()
    return out


def max_over(ws: int, dev, x: float) -> float:
    if ws == 1:
        return x
    t = torch.tensor([x], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def load_pmc_key(key: str) -> dict:
    """Per-phase HBM bytes and VALU figures per launch from the committed PMC passes (tools/pmc_traffic.py), keyed by
    workload ("{N}x{W}x{H}", "-sparse" for the non-saturating scene)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        return json.load(open(path)).get(key, {})
    except Exception:  # noqa: BLE001
        return {}


def load_pmc(n: int, W: int, H: int):
    return load_pmc_key(f"{n}x{W}x{H}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); > 1 without a launcher relaunches under torch.distributed.run")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=8)
    # --gaussians: the same, spelled so that torch.distributed.run's own argparse (which matches option prefixes
    # anywhere on the command line) does not read `--n` as an abbreviation of its --nnodes / --nproc-per-node
    ap.add_argument("--n", "--gaussians", dest="n", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--views", type=int, default=8)
    ap.add_argument("--opacity-mean", type=float, default=0.0,
                    help="raw opacity ~ N(mean, 1.5): -2 is the sweep's non-saturating scene (profiling runs)")
    ap.add_argument("--consensus-interval", type=int, default=200)
    ap.add_argument("--shared-frac", type=float, default=0.2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-train-step", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds per CPU-baseline leg")
    ap.add_argument("--no-admm", action="store_true", help="skip the ADMM block-trainer leg")
    ap.add_argument("--admm-rounds", type=int, default=1, help="timed ADMM rounds (each: interval local steps)")
    ap.add_argument("--admm-interval", type=int, default=200, help="local steps per round (urban3d_admm.yaml:44)")
    ap.add_argument("--admm-pre", type=int, default=200,
                    help="pre-phase iterations (densify_end_iter of the ADMM leg's run; interval chunks)")
    ap.add_argument("--launch-check", action="store_true",
                    help="plumbing check, no GPU: every rank joins a gloo group, all_reduces its rank and rank 0 "
                         "prints the world it saw (tests/test_bench_launch.py)")
    ap.add_argument("--no-sweep", action="store_true", help="skip the other workloads (1e5, 5e6, 4K, sparse scene)")
    ap.add_argument("--sweep-only", default=None, help="comma-separated subset of the sweep's workload names")
    ap.add_argument("--no-reference-k", action="store_true",
                    help="skip the untimed depth-prefix-off forwards (profiling runs: keeps kernel averages clean)")
    args = ap.parse_args()
    # nothing has touched the GPU yet: the launcher runs as a child process (never an exec from this process)
    cmd = relaunch_command(args.gpus, sys.argv[1:], os.environ)
    if cmd is not None:
        import subprocess
        print("[bench] launching " + " ".join(cmd), file=sys.stderr)
        sys.exit(subprocess.call(cmd))

    ws, rank, local = dist_env()
    check_world(args.gpus, ws)
    if args.launch_check:
        if ws > 1:
            dist.init_process_group("gloo")
        t = torch.tensor([rank], dtype=torch.int64)
        if ws > 1:
            dist.all_reduce(t)
        if rank == 0:
            print(json.dumps({"n_gpus": ws, "rank_sum": int(t.item()), "gpus_arg": args.gpus}))
        if ws > 1:
            dist.destroy_process_group()
        return
    # one rank per GPU over RCCL ("nccl" on ROCm).  DOGS_DIST_BACKEND=gloo + DOGS_BENCH_SHARE_DEVICE=1 rehearse the
    # multi-rank control flow with several ranks on one GPU (RCCL needs distinct devices).
    backend = os.environ.get("DOGS_DIST_BACKEND", "nccl")
    if os.environ.get("DOGS_BENCH_SHARE_DEVICE") == "1":
        local = local % max(torch.cuda.device_count(), 1)
    if ws > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local if ws > 1 else 0)
    import dogs_amd._lib as L
    L.load()

    n, W, H = args.n, args.width, args.height
    seed = 1234 + rank
    from dogs_amd.synthetic import make_scene
    s = make_scene(n, W, H, seed=seed, opacity_mean=args.opacity_mean).to(dev)
    yaws = view_yaws(args.views)
    cams = make_cameras(W, H, yaws, dev)
    g = torch.Generator().manual_seed(seed + 99)
    grad_color = torch.randn((3, H, W), generator=g).to(dev)
    grad_inv = torch.zeros((1, H, W), device=dev)
    views = Views(s, cams, grad_color, grad_inv, dev)
    with torch.cuda.device(dev):
        L.adaptive_capacity(W, H, reset=True)   # every run starts cold; the warmup views let it settle

    cons = None
    if ws > 1:
        from dogs_amd.admm import BlockConsensus
        # block k holds global ids [k*n(1-f), k*n(1-f)+n): its last f*n are the next block's first f*n
        stride = int(round(n * (1.0 - args.shared_frac)))
        gidx = torch.arange(rank * stride, rank * stride + n, device=dev)
        num_global = stride * (ws - 1) + n
        cons = BlockConsensus(gidx, num_global, device=dev)
        cparams = (s.means3D, s.dc, s.sh, s.raw_scales.to(dev), s.raw_rotations.to(dev), s.raw_opacities.to(dev))

    def max_over_ranks(x):
        if ws == 1:
            return x
        t = torch.tensor([x], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    for _ in range(args.warmup):
        views.step()
    if cons is not None:
        cons.consensus(cparams)  # untimed: the first exchange carries one-time buffer and communicator setup
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step_t = []
    for _ in range(args.steps):
        ts = time.perf_counter()
        views.step()
        step_t.append(time.perf_counter() - ts)
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    st = sorted(step_t)
    print(f"[bench rank {rank}] host time per step (launch + forward sync): min {st[0] * 1e3:.3f} "
          f"median {st[len(st) // 2] * 1e3:.3f} max {st[-1] * 1e3:.3f} ms", file=sys.stderr)
    # The consensus runs once per consensus_interval steps (urban3d_admm.yaml:44: 200).  It is timed on its own,
    # barrier-bracketed like the steps, and its cost is added in that proportion (a K-step window either misses it
    # or, holding one whole exchange, would overweight it K/interval-fold).
    cons_s = 0.0
    if cons is not None:
        dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        cons.consensus(cparams)
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        cons_s = max_over_ranks(time.perf_counter() - t1)
        elapsed += cons_s * args.steps / args.consensus_interval
    view_ms = elapsed / args.steps * 1e3
    with torch.cuda.device(dev):
        cap = L.adaptive_capacity(W, H)

    # ---- untimed per-view figures, then one profiled pass over the views: per-phase hipEvent durations on the stream
    # the kernels run on
    HW = W * H
    vstats = []
    for k, y in enumerate(yaws):
        r = views.stats(k, reference_k=not args.no_reference_k)
        r.update(view=k, yaw=round(y, 3), N=n, HW=HW)
        vstats.append(r)
    pmc = load_pmc_key(f"{n}x{W}x{H}" + ("-sparse" if args.opacity_mean != 0.0 else ""))
    pp = phase_profile(views, yaws, vstats, pmc)
    phase_ms, phase_b, dom = pp["phase_ms_raw"], pp["phase_b_raw"], pp["dominant"]
    dom_ms, dom_bytes = phase_ms[dom], phase_b[dom]
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    view_bytes = pp["view_bytes"]
    K_mean = float(np.mean([r["K"] for r in vstats])) if not args.no_reference_k else float("nan")
    ref_bytes = reference_view_bytes(n, int(K_mean), HW) if K_mean == K_mean else float("nan")

    traffic = pmc.get(dom, {}).get("hbm_bytes") if isinstance(pmc.get(dom), dict) else None
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": dom,
            "kernel_ms": round(dom_ms, 4), "kernel_bytes": round(dom_bytes),
            "view_bytes": round(view_bytes), "view_achieved_GBs": round(view_bytes / (view_ms * 1e-3) / 1e9, 1),
            "view_frac": round(view_bytes / (view_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "phase_bytes": {k: round(v) for k, v in phase_b.items() if v > 0},
            "valu": pp["valu"], "phase_hbm_frac": pp["phase_hbm_frac"],
            "reference_equivalent": {
                "formula": "856 N + 172 K + 64 HW (SURVEY.md 8(d), the reference's full per-tile lists)",
                "view_bytes": round(ref_bytes) if ref_bytes == ref_bytes else None,
                "K_mean": round(K_mean) if K_mean == K_mean else None,
                "view_frac": (round(ref_bytes / (view_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                              if ref_bytes == ref_bytes else None)}}

    train = None
    if not args.no_train_step and ws == 1:
        ts = TrainStep(s, cams, dev, seed)
        for _ in range(len(cams)):
            ts.step()
        torch.cuda.synchronize()
        tt = time.perf_counter()
        nts = max(2 * len(cams), args.steps // 2)
        host = []
        w0 = int(L.load().dg_host_wait_ns())
        for _ in range(nts):
            th = time.perf_counter()
            ts.step()
            host.append(time.perf_counter() - th)
        torch.cuda.synchronize()
        tms = (time.perf_counter() - tt) / nts * 1e3
        host_ms = float(np.median(host)) * 1e3
        wait_ms = (int(L.load().dg_host_wait_ns()) - w0) / nts / 1e6
        nstep = ts.native()
        route_ms = {}
        # the default route (activation backward folded into the update) and the unfused one, interleaved three
        # times (the box drifts by a few % over a run); the best of each
        for _rep in range(3):
            for route, env in (("unfused", "DG_TRAIN_UNFUSED"), ("folded", None)):
                if env:
                    os.environ[env] = "1"
                try:
                    for _ in range(len(cams)):
                        nstep()
                    torch.cuda.synchronize()
                    tt = time.perf_counter()
                    for _ in range(nts):
                        nstep()
                    torch.cuda.synchronize()
                    ms = round((time.perf_counter() - tt) / nts * 1e3, 4)
                    route_ms[route] = min(route_ms.get(route, ms), ms)
                finally:
                    if env:
                        del os.environ[env]
        nms = route_ms["folded"]
        dms, n_after = ts.densify()
        masked = masked_iteration_leg(s, cams, dev, seed)
        train = {"views_per_s": round(1e3 / tms, 2), "ms_per_step": round(tms, 3),
                 "includes": "activations + raster fwd/bwd + L1 + fused-SSIM fwd/bwd + scale regulariser + "
                             "densification stats + SparseGaussianAdam (one launch), cycling the view batch; "
                             "autograd route (the drop-in API)",
                 "host_ms_per_step": round(host_ms, 3),
                 "host_wait_ms_per_step": round(wait_ms, 3),
                 "host_note": "median host time per autograd-route step (Python + autograd + launches, and the "
                              "forward's one wait for the phase-1 counters); above ms_per_step the GPU waits on it. "
                              "host_wait_ms_per_step: the mean of that wait (dg_host_wait_ns), i.e. host time that "
                              "is the GPU's, not Python's",
                 "native": {"views_per_s": round(1e3 / nms, 2), "ms_per_step": round(nms, 3),
                            "route": "dg_train_step (dogs_amd.train_step): the same iteration in one C call, the "
                                     "activation backward folded into the optimizer update",
                            "routes_ms": route_ms},
                 "densify_and_prune_ms": round(dms, 3), "gaussians_after_densify": n_after,
                 "masked_config2": masked}

    sweep = None
    if not args.no_sweep and ws == 1:
        sweep = sweep_leg(dev, yaws, seed, only=args.sweep_only.split(",") if args.sweep_only else None)

    admm = None
    if not args.no_admm:
        del views
        torch.cuda.empty_cache()
        admm = admm_leg(args, ws, rank, dev, n, W, H)

    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(n, W, H, seed, yaws, budget_s=args.cpu_budget)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(args.steps * ws / elapsed, 3),
            "unit": "views/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(view_ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic (BASELINE.md §2 generator, seed 1234+rank; {len(yaws)} seeded yaw views; random "
                    "dL/dcolor, zero dL/dinvdepth)",
            "config": {"workload": f"synthetic {W}x{H}, {n} Gaussians/rank, SH3, raster fwd+bwd per view, "
                                   f"{len(yaws)}-view yaw batch",
                       "width": W, "height": H, "gaussians_per_rank": n, "sh_degree": 3,
                       "adaptive_capacity_per_tile": cap,
                       "consensus_interval": args.consensus_interval if ws > 1 else None,
                       "consensus_ms": round(cons_s * 1e3, 3) if ws > 1 else None,
                       "shared_gaussians": (cons.num_shared if cons is not None else 0),
                       "parallelism": f"admm-blocks x{ws}" if ws > 1 else "single"},
            "views": [{k: r[k] for k in ("view", "yaw", "num_rendered", "K", "e1", "e2", "unfinished_tiles",
                                         "visible_gaussians", "binned_gaussians", "live_gaussians")} for r in vstats],
            "roofline": roof,
            "phases_ms": {k: round(v, 4) for k, v in sorted(phase_ms.items(), key=lambda kv: -kv[1])},
            "phases_note": "per-phase hipEvent times from a separate, untimed pass over the same views (event records "
                           "between phases serialise the queue, so their sum exceeds ms_per_step)",
            "cpu_baseline": cpu,
            "train_step": train,
            "sweep": sweep,
            "admm": admm,
        }
        print(json.dumps(line))
    if ws > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
