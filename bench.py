"""bench.py -- train views/sec (fwd+bwd raster) @1080p, 1e6 Gaussians; 1/2/4/8-GPU ADMM scaling.

One step = one view per rank: _C.rasterize_gaussians + _C.rasterize_gaussians_backward on the synthetic
1080p scene of BASELINE.md §2 (SH degree 3, AA off, fixed random dL/dcolor, zero dL/dinvdepth), inputs
resident in HBM.  With N > 1 ranks (torch.distributed.run, one GPU each, RCCL) every rank trains its own
scene block and the ADMM consensus all_reduce of the shared Gaussians runs every --consensus-interval
steps and at least once inside the timed region.  value = views of all ranks / max-over-ranks time.

Also reported on the same JSON line:
  roofline      per-phase hipEvent timing of one extra profiled step; algorithmic bytes per phase from
                SURVEY.md §8(d) (B_view = 856 N + 172 K + 64 HW); `traffic` from the committed rocprofv3
                PMC summary of the same command when present (profiles/), else null
  cpu_baseline  the CPU oracle (oracle/gs_oracle.c restating the reference kernels) on one view of the
                same scene, rank 0 at N = 1 only
  train_step    secondary figure: fwd + L1 + fused-SSIM fwd/bwd + bwd + densification stats + SparseGaussianAdam
                (6 groups, one launch), and one densify_and_prune timed on the trained state
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "train views/sec (fwd+bwd raster) @1080p, 1e6 Gaussians; 1/2/4/8-GPU ADMM scaling"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def phase_bytes(phase: str, N: int, K: int, HW: int) -> float:
    """Algorithmic bytes per launch of each phase (DESIGN.md 'Roofline'), with K the reference's
    precise instance count (its full per-tile lists), whatever this build bins."""
    return {
        "preprocess": 284.0 * N,            # 236 B params read + 48 B geometry written
        "prefix_cut": 8.0 * N,              # depth histogram: key + count per Gaussian
        "count_scan": 8.0 * N,
        "tile_dsort": 0.0,                  # implementation overhead: per-tile depth order of the binned lists
        "emit": 36.0 * N + 12.0 * K,
        "tile_sort": 24.0 * K,
        "ranges": 8.0 * K,
        "render_fwd": 44.0 * K + 24.0 * HW,
        "flag_clear": 0.0,
        "render_bwd": 84.0 * K + 40.0 * HW,
        "record_sum": 0.0,                  # implementation overhead (per-instance records -> sums)
        "phase2_count": 0.0,                # depth-prefix binning, phase 2 (only when tiles were left unfinished)
        "phase2_bin": 0.0,
        "render_fwd2": 0.0,
        "gauss_bwd": 528.0 * N,
    }.get(phase, 0.0)


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def make_inputs(n, W, H, seed, dev):
    from dogs_amd.synthetic import make_scene
    s = make_scene(n, W, H, seed=seed).to(dev)
    g = torch.Generator().manual_seed(seed + 99)
    grad_color = torch.randn((3, H, W), generator=g).to(dev)
    grad_inv = torch.zeros((1, H, W), device=dev)
    return s, grad_color, grad_inv


class View:
    """One fwd+bwd raster step through the drop-in `_C` table."""

    def __init__(self, s, grad_color, grad_inv, dev):
        from dogs_amd.diff_gaussian_rasterization import _C
        self._C = _C
        self.s, self.gc, self.gi, self.dev = s, grad_color, grad_inv, dev
        self.c = s.camera
        self.bg = torch.zeros(3, device=dev)
        self.e = torch.empty(0, device=dev)
        self.last = None

    def forward(self):
        s, c, e = self.s, self.c, self.e
        return self._C.rasterize_gaussians(self.bg, s.means3D, e, s.opacities, s.scales, s.rotations, 1.0, e,
                                           c.world_to_camera, c.projective_matrix, c.tanfovx, c.tanfovy, c.height,
                                           c.width, s.dc, s.sh, 3, c.camera_center, False, False, False)

    def reference_instances(self):
        """The reference's precise instance count (its full per-tile lists): one untimed forward with
        depth-prefix binning off.  The §8(d) byte formula is written in terms of it."""
        old = self._C.set_prefix_per_tile(-1)
        try:
            self.last_out = self.forward()
            return self.binned_instances()
        finally:
            self._C.set_prefix_per_tile(old)

    def step(self):
        s, c, e = self.s, self.c, self.e
        out = self._C.rasterize_gaussians(self.bg, s.means3D, e, s.opacities, s.scales, s.rotations, 1.0, e,
                                          c.world_to_camera, c.projective_matrix, c.tanfovx, c.tanfovy, c.height,
                                          c.width, s.dc, s.sh, 3, c.camera_center, False, False, False)
        g = self._C.rasterize_gaussians_backward(self.bg, s.means3D, out[4], e, s.opacities, s.scales, s.rotations,
                                                 1.0, e, c.world_to_camera, c.projective_matrix, c.tanfovx,
                                                 c.tanfovy, self.gc, s.dc, s.sh, self.gi, 3, c.camera_center,
                                                 out[5], out[0], out[6], out[7], out[1], out[8], False, False)
        self.last = (out[0], out[1])
        self.last_out = out
        return out, g

    def binned_instances(self):
        import ctypes as C
        import dogs_amd._lib as L
        v = C.c_int64(-1)
        if not hasattr(L.load(), "dg_binned_instances"):
            return -1
        L.check(L.load().dg_binned_instances(self.last_out[5].data_ptr(), int(self.s.means3D.shape[0]), C.byref(v),
                                             L.stream_of(self.dev)))
        return int(v.value)


class TrainStep:
    """Training iteration of GaussianSplatTrainer.train_iteration (gaussian_trainer.py:324-513) before
    densify_end_iter, without the periodic densify_and_prune: activations, raster, L1 + fused-SSIM, backward, the
    view's densification statistics (:433-438) and SparseGaussianAdam.step(visible, N) -- the last two in one
    launch.  densify() times one densify_and_prune (dogs_amd.densify) on the trained state."""

    def __init__(self, s, dev, seed):
        from dogs_amd.diff_gaussian_rasterization import (GaussianRasterizationSettings, GaussianRasterizer,
                                                          SparseGaussianAdam)
        from dogs_amd.activations import activate
        from dogs_amd.fused_ssim import fused_ssim
        from dogs_amd.loss import clamp_l1
        self.activate = activate
        self.clamp_l1 = clamp_l1
        self.fused_ssim = fused_ssim
        self.s = s
        c = s.camera
        self.rs = GaussianRasterizationSettings(c.height, c.width, c.tanfovx, c.tanfovy, torch.zeros(3, device=dev),
                                                1.0, c.world_to_camera, c.projective_matrix, 3, c.camera_center,
                                                False, False, False, 0.0)
        self.rast = GaussianRasterizer(self.rs)
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
        g = torch.Generator().manual_seed(seed + 7)
        self.gt = torch.rand((3, c.height, c.width), generator=g).to(dev)
        N = s.means3D.shape[0]
        self.stats = {"max_radii2D": torch.zeros(N, device=dev), "grad_accum": torch.zeros((N, 1), device=dev),
                      "denom": torch.zeros((N, 1), device=dev)}

    def step(self):
        p = self.params
        m2d = torch.zeros_like(p["xyz"], requires_grad=True)
        # get_opacity / get_scaling / get_quaternion (sigmoid, exp, normalize) fused in one launch each way
        opac, scales, rots = self.activate(p["opacity"], p["scaling"], p["quaternion"])
        img, radii, _ = self.rast(means3D=p["xyz"], means2D=m2d, opacities=opac, dc=p["f_dc"], shs=p["f_rest"],
                                  scales=scales, rotations=rots)
        img, l1 = self.clamp_l1(img, self.gt)  # render()'s clamp + the L1 term, one launch each way
        ssim = self.fused_ssim(img.unsqueeze(0), self.gt.unsqueeze(0))
        loss = 0.8 * l1 + 0.2 * (1.0 - ssim)
        loss.backward()
        vis = radii > 0
        self.opt.step(vis, radii.shape[0], stats=dict(self.stats, radii=radii, dmeans2D=m2d.grad))
        self.opt.zero_grad(set_to_none=True)

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


def cpu_baseline(n, W, H, seed):
    """Oracle fwd+bwd of one view of the same scene on this host (1 core): the reference has no CPU
    rasterizer, so this is the CPU restatement of its kernels."""
    from oracle import oracle as O
    from dogs_amd.synthetic import make_scene
    O.build()
    s = make_scene(n, W, H, seed=seed)
    c = s.camera
    g = torch.Generator().manual_seed(seed + 99)
    gc = torch.randn((3, H, W), generator=g).numpy()
    t0 = time.perf_counter()
    _, _, _, st = O.forward(s.means3D.numpy(), s.opacities.numpy(), c.world_to_camera.numpy(),
                            c.projective_matrix.numpy(), c.camera_center.numpy(), c.tanfovx, c.tanfovy, H, W,
                            np.zeros(3, np.float32), dc=s.dc.numpy(), sh=s.sh.numpy(), scales=s.scales.numpy(),
                            rotations=s.rotations.numpy())
    st.backward(gc)
    dt = time.perf_counter() - t0
    try:
        model = [l for l in open("/proc/cpuinfo") if l.startswith("model name")][0].split(":", 1)[1].strip()
    except Exception:  # noqa: BLE001
        model = "unknown"
    return {"value": round(1.0 / dt, 5), "unit": "views/s", "cores": 1, "kind": "port",
            "sample": f"1 view fwd+bwd of the same {W}x{H} / {n} Gaussian scene, 1 thread ({model})",
            "seconds": round(dt, 3)}


def load_traffic(phase: str, n: int, W: int, H: int):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
        e = d.get(f"{n}x{W}x{H}", {}).get(phase)
        return None if e is None else float(e)
    except Exception:  # noqa: BLE001
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--consensus-interval", type=int, default=200)
    ap.add_argument("--shared-frac", type=float, default=0.2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-train-step", action="store_true")
    args = ap.parse_args()

    ws, rank, local = dist_env()
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
    s, gc, gi = make_inputs(n, W, H, seed, dev)
    view = View(s, gc, gi, dev)

    cons = None
    if ws > 1:
        from dogs_amd.admm import BlockConsensus
        # block k holds global ids [k*n(1-f), k*n(1-f)+n): its last f*n are the next block's first f*n
        stride = int(round(n * (1.0 - args.shared_frac)))
        gidx = torch.arange(rank * stride, rank * stride + n, device=dev)
        num_global = stride * (ws - 1) + n
        cons = BlockConsensus(gidx, num_global, device=dev)
        cparams = (s.means3D, s.dc, s.sh, s.raw_scales.to(dev), s.raw_rotations.to(dev), s.raw_opacities.to(dev))

    def one(i):
        view.step()
        if cons is not None and ((i + 1) % args.consensus_interval == 0):
            cons.consensus(cparams)

    def max_over_ranks(x):
        if ws == 1:
            return x
        t = torch.tensor([x], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    for i in range(args.warmup):
        one(i)
    if cons is not None:
        cons.consensus(cparams)  # untimed: the first exchange carries one-time buffer and communicator setup
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step_t = []
    for i in range(args.steps):
        ts = time.perf_counter()
        one(i)
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
    num_rendered = view.last[0]
    K_binned = view.binned_instances()
    K = view.reference_instances()

    # ---- one profiled step: per-phase hipEvent durations on the stream the kernels run on
    L.profile_enable(True)
    view.step()
    torch.cuda.synchronize()
    prof = L.profile_collect()
    L.profile_enable(False)
    HW = W * H
    phases = {k: round(v[0], 4) for k, v in sorted(prof.items(), key=lambda kv: -kv[1][0])}
    dom = max(prof.items(), key=lambda kv: kv[1][0] if phase_bytes(kv[0], n, K, HW) > 0 else -1)[0]
    dom_ms = prof[dom][0] / max(prof[dom][1], 1)
    dom_bytes = phase_bytes(dom, n, K, HW)
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    b_view = 856.0 * n + 172.0 * K + 64.0 * HW
    view_ms = elapsed / args.steps * 1e3
    traffic = load_traffic(dom, n, W, H)

    train = None
    if not args.no_train_step and ws == 1:
        ts = TrainStep(s, dev, seed)
        for _ in range(3):
            ts.step()
        torch.cuda.synchronize()
        tt = time.perf_counter()
        nts = max(5, args.steps // 2)
        for _ in range(nts):
            ts.step()
        torch.cuda.synchronize()
        tms = (time.perf_counter() - tt) / nts * 1e3
        dms, n_after = ts.densify()
        train = {"views_per_s": round(1e3 / tms, 2), "ms_per_step": round(tms, 3),
                 "includes": "activations + raster fwd/bwd + L1 + fused-SSIM fwd/bwd + densification stats + "
                             "SparseGaussianAdam (one launch)",
                 "densify_and_prune_ms": round(dms, 3), "gaussians_after_densify": n_after}

    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(n, W, H, seed)

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
            "data": "synthetic (BASELINE.md §2 generator, seed 1234+rank; random dL/dcolor, zero dL/dinvdepth)",
            "config": {"workload": f"synthetic {W}x{H}, {n} Gaussians/rank, SH3, raster fwd+bwd per view",
                       "width": W, "height": H, "gaussians_per_rank": n, "sh_degree": 3,
                       "num_rendered": int(num_rendered), "instances_K": int(K),
                       "instances_binned": int(K_binned),
                       "consensus_interval": args.consensus_interval if ws > 1 else None,
                       "consensus_ms": round(cons_s * 1e3, 3) if ws > 1 else None,
                       "shared_gaussians": (cons.num_shared if cons is not None else 0),
                       "parallelism": f"admm-blocks x{ws}" if ws > 1 else "single"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": dom,
                         "kernel_ms": round(dom_ms, 4), "kernel_bytes": dom_bytes,
                         "view_bytes": b_view, "view_achieved_GBs": round(b_view / (view_ms * 1e-3) / 1e9, 1),
                         "view_frac": round(b_view / (view_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "phases_ms": phases,
            "cpu_baseline": cpu,
            "train_step": train,
        }
        print(json.dumps(line))
    if ws > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
