"""BASELINE config 2 at its own schedule: the mipnerf360 'garden' single-GPU trainer, full 30k-iteration run at 1080p.

The schedule is the reference's config/gaussian_splatting/mipnerf360.yaml (:25 max_iterations 30000, :74-77 densify
from 500 to 15000 every 100, opacity reset every 3000; the SH degree raised every 1000 iterations,
gaussian_trainer.py:328; geometry.mask on with lambda_mask 0), read from the committed parse of that file
(tests/golden/reference_configs.json) through GSTrainConfig.from_reference, and the loop is
dogs_amd.trainer.GaussianSplatTrainer (gaussian_trainer.py:324-513) on its default native route.

There is no dataset on the box, so the scene is synthetic (BASELINE §2's generator, dogs_amd.synthetic): the targets
are 1920 x 1080 renders of a 1e6-Gaussian ground-truth scene from 24 cameras spread over a 3-unit baseline (so the
camera radius that sets spatial_lr_scale is not zero), every 8th view held out as the test split (the dataset's
val_interval 8), and the model starts from a 100k-point subset of the true centres with their colours
(init_from_colmap_pcd, like an SfM cloud).

Recorded (JSON): every 1000 iterations the train / test PSNR, the Gaussian count, the active SH degree, wall-clock,
peak device memory and whether every parameter is finite; the events the loop ran; the totals.

    python tools/train_30k.py --out gpurun_out/t30k/run.json
    python tools/train_30k.py --compare 2000 --out gpurun_out/t30k/routes.json   # native vs autograd route
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

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cameras(W, H, fx, n, dev):
    """n cameras with centres on x in [-1.5, 1.5] (y alternating +-0.2) and yaws in [-4, 4] degrees, all facing +z."""
    from dogs_amd.camera import make_camera
    cams = []
    for i in range(n):
        t = i / max(n - 1, 1)
        cx, cy = -1.5 + 3.0 * t, 0.2 * (1 if i % 2 else -1)
        yaw = math.radians(-4.0 + 8.0 * ((i * 7) % n) / max(n - 1, 1))
        c, s = math.cos(yaw), math.sin(yaw)
        R = torch.tensor([[c, 0.0, -s], [0.0, 1.0, 0.0], [s, 0.0, c]])
        w2c = torch.eye(4)
        w2c[:3, :3] = R
        w2c[:3, 3] = -R @ torch.tensor([cx, cy, 0.0])
        cam = make_camera(W, H, fx, fx, world_to_camera=w2c)
        cams.append(cam.to(dev))
    return cams


@torch.no_grad()
def render_raw(raw, cam, sh_degree, dev):
    from dogs_amd.diff_gaussian_rasterization import _C
    e = torch.empty(0, device=dev)
    out = _C.rasterize_gaussians(torch.zeros(3, device=dev), raw["xyz"], e, torch.sigmoid(raw["opacity"]),
                                 torch.exp(raw["scaling"]), torch.nn.functional.normalize(raw["quaternion"]), 1.0, e,
                                 cam.world_to_camera, cam.projective_matrix, cam.tanfovx, cam.tanfovy, cam.height,
                                 cam.width, raw["features_dc"], raw["features_rest"], sh_degree, cam.camera_center,
                                 False, False, False)
    return out[2].clamp(0, 1)


def model_raw(m):
    return {"xyz": m._xyz.detach(), "features_dc": m._features_dc.detach(),
            "features_rest": m._features_rest.detach(), "opacity": m._opacity.detach(),
            "scaling": m._scaling.detach(), "quaternion": m._quaternion.detach()}


def psnr(a, b):
    return -10.0 * math.log10(max(float(((a - b) ** 2).mean()), 1e-20))


def problem(dev, n_true, n_init, W, H, fx, views, seed=21):
    from dogs_amd.gaussian_model import GaussianSplatModel
    from dogs_amd.synthetic import make_scene
    s = make_scene(n_true, W, H, fx=fx, fy=fx, seed=seed)
    true = {"xyz": s.means3D.to(dev), "features_dc": s.dc.to(dev), "features_rest": s.sh.to(dev),
            "scaling": s.raw_scales.to(dev).contiguous(), "quaternion": s.raw_rotations.to(dev).contiguous(),
            "opacity": s.raw_opacities.to(dev).contiguous()}
    cams = cameras(W, H, fx, views, dev)
    gts = [render_raw(true, c, 3, dev).contiguous() for c in cams]
    del true
    g = torch.Generator().manual_seed(5)
    pick = torch.randperm(n_true, generator=g)[:n_init]
    pts = s.means3D[pick].numpy()
    cols = (s.dc[pick, 0] * 0.28209479177387814 + 0.5).clamp(0, 1).numpy()
    m = GaussianSplatModel(3, 0.01, dev)
    m.init_from_colmap_pcd(pts, cols)
    return m, cams, gts


def split(cams, gts):
    test = [i for i in range(len(cams)) if i % 8 == 0]
    train = [i for i in range(len(cams)) if i % 8 != 0]
    return train, test


def evaluate(m, cams, gts, idx, dev):
    raw = model_raw(m)
    return float(np.mean([psnr(render_raw(raw, cams[i], m.active_sh_degree, dev), gts[i]) for i in idx]))


def finite(m) -> bool:
    return all(bool(torch.isfinite(t).all()) for t in model_raw(m).values())


def reference_cfg(**over):
    from dataclasses import replace
    from dogs_amd.trainer import GSTrainConfig
    with open(os.path.join(ROOT, "tests", "golden", "reference_configs.json")) as f:
        d = json.load(f)["mipnerf360.yaml"]
    cfg = GSTrainConfig.from_reference(d)
    return replace(cfg, **over) if over else cfg


def log(msg):
    print(msg, flush=True)


def run_full(args, dev):
    from dogs_amd.trainer import GaussianSplatTrainer
    over = {"max_iterations": args.iterations} if args.iterations else {}
    if args.mask == "off":
        over["mask"] = False
    cfg = reference_cfg(**over)
    m, cams, gts = problem(dev, args.n_true, args.n_init, args.width, args.height, args.fx, args.views)
    tr_idx, te_idx = split(cams, gts)
    torch.manual_seed(0)
    tr = GaussianSplatTrainer(m, [cams[i] for i in tr_idx], [gts[i] for i in tr_idx], cfg, device=dev, seed=42,
                              native=True)
    rec = {"workload": "mipnerf360.yaml schedule (config 2), synthetic 1e6-Gaussian 1080p scene",
           "config": {k: getattr(cfg, k) for k in ("max_iterations", "densify_start_iter", "densify_end_iter",
                                                   "densification_interval", "opacity_reset_interval",
                                                   "densify_grad_threshold", "sh_increase_interval", "mask",
                                                   "lambda_mask", "lambda_dssim", "lambda_scale", "max_sh_degree")},
           "spatial_lr_scale": tr.spatial_lr_scale, "n_true": args.n_true, "n_init": args.n_init,
           "image": [args.width, args.height], "train_views": len(tr_idx), "test_views": len(te_idx),
           "data": "synthetic", "device": torch.cuda.get_device_name(dev), "trace": []}
    torch.cuda.reset_peak_memory_stats(dev)
    p_tr, p_te = evaluate(m, cams, gts, tr_idx, dev), evaluate(m, cams, gts, te_idx, dev)
    rec["trace"].append({"iteration": 0, "train_psnr": p_tr, "test_psnr": p_te, "gaussians": m.num_gaussians,
                         "sh_degree": m.active_sh_degree, "wall_s": 0.0, "finite": finite(m)})
    log(json.dumps(rec["trace"][-1]))
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    train_s = 0.0
    every = args.every
    while tr.iteration < cfg.max_iterations:
        ts = time.perf_counter()
        for _ in range(min(every, cfg.max_iterations - tr.iteration)):
            tr.train_iteration()
            if tr.iteration % 100 == 0:
                log(f"iteration {tr.iteration} gaussians {m.num_gaussians} elapsed {time.perf_counter() - t0:.1f} s")
        tr.sync()
        torch.cuda.synchronize(dev)
        train_s += time.perf_counter() - ts
        it = tr.iteration
        p_tr, p_te = evaluate(m, cams, gts, tr_idx, dev), evaluate(m, cams, gts, te_idx, dev)
        ok = finite(m)
        e = {"iteration": it, "train_psnr": p_tr, "test_psnr": p_te, "gaussians": m.num_gaussians,
             "sh_degree": m.active_sh_degree, "wall_s": time.perf_counter() - t0, "train_s": train_s,
             "peak_mem_gb": torch.cuda.max_memory_allocated(dev) / 2 ** 30, "finite": ok,
             "loss": float(tr.loss()) if tr.loss() is not None else None}
        rec["trace"].append(e)
        log(json.dumps(e))
        if not ok:
            log("non-finite parameters: stopping")
            break
    ev = [(lg.iteration, lg.events) for lg in tr.logs if lg.events]
    rec["events"] = {"densify": [i for i, e in ev if "densify" in e],
                     "reset_opacity": [i for i, e in ev if "reset_opacity" in e],
                     "prune": [i for i, e in ev if "prune" in e]}
    rec["routes"] = {"native": sum(lg.route == "native" for lg in tr.logs),
                     "autograd": sum(lg.route == "autograd" for lg in tr.logs)}
    counts = [lg.num_gaussians for lg in tr.logs]
    rec["count_changes_outside_densify"] = [i + 1 for i in range(1, len(counts))
                                            if counts[i] != counts[i - 1] and "densify" not in tr.logs[i].events]
    rec["gaussians_max"] = max(counts)
    rec["total"] = {"iterations": tr.iteration, "wall_s": time.perf_counter() - t0, "train_s": train_s,
                    "ms_per_iteration": 1e3 * train_s / max(tr.iteration, 1),
                    "peak_mem_gb": torch.cuda.max_memory_allocated(dev) / 2 ** 30,
                    "all_finite": all(e["finite"] for e in rec["trace"]),
                    "psnr_first_last": [rec["trace"][0]["test_psnr"], rec["trace"][-1]["test_psnr"]]}
    return rec


def run_compare(args, dev):
    """The native route against the autograd route (every iteration through render() + SparseGaussianAdam, as the
    reference's trainer calls the drop-in API) over the first `compare` iterations of the same schedule, same seeds."""
    from dogs_amd.trainer import GaussianSplatTrainer
    cfg = reference_cfg()
    out = {"iterations": args.compare, "workload": "mipnerf360.yaml schedule, first iterations, both routes",
           "routes": {}}
    states = []
    for native in (True, False):
        m, cams, gts = problem(dev, args.n_true, args.n_init, args.width, args.height, args.fx, args.views)
        tr_idx, te_idx = split(cams, gts)
        g = torch.Generator(device=dev).manual_seed(7)
        torch.manual_seed(0)    # the appearance embedding's initial weights: the same for both routes
        tr = GaussianSplatTrainer(m, [cams[i] for i in tr_idx], [gts[i] for i in tr_idx], cfg, device=dev, seed=42,
                                  native=native, normal=lambda mean, std: torch.normal(mean, std, generator=g))
        losses, counts = [], []
        t0 = time.perf_counter()
        for i in range(args.compare):
            tr.train_iteration()
            losses.append(float(tr.loss()))
            counts.append(m.num_gaussians)
            if (i + 1) % 500 == 0:
                log(f"{'native' if native else 'autograd'} {i + 1} loss {losses[-1]:.5f} gaussians {counts[-1]}")
        tr.sync()
        wall = time.perf_counter() - t0
        st = {f"param.{k}": v.detach().clone() for k, v in m.params().items()}
        for g_ in tr.optimizer.param_groups:
            o_ = tr.optimizer.state[g_["params"][0]]
            st[f"m.{g_['name']}"], st[f"v.{g_['name']}"] = o_["exp_avg"].clone(), o_["exp_avg_sq"].clone()
        st["net"] = torch.cat([p_.detach().reshape(-1) for p_ in tr.mask.parameters()]) if tr.mask is not None else None
        states.append(st)
        out["routes"]["native" if native else "autograd"] = {
            "losses": losses, "counts": counts, "wall_s": wall, "finite": finite(m),
            "test_psnr": evaluate(m, cams, gts, te_idx, dev), "train_psnr": evaluate(m, cams, gts, tr_idx, dev)}
        del tr, m, gts
        torch.cuda.empty_cache()
    a, b = out["routes"]["native"], out["routes"]["autograd"]
    la, lb, ca, cb = map(np.asarray, (a["losses"], b["losses"], a["counts"], b["counts"]))
    first = int(np.argmax(ca != ca[0])) if np.any(ca != ca[0]) else len(ca)
    out["first_densify_index"] = first
    out["max_rel_loss_diff_before_first_densify"] = float(np.max(np.abs(la[:first] - lb[:first]) / lb[:first]))
    dens = [i for i in range(1, len(ca)) if ca[i] != ca[i - 1] or cb[i] != cb[i - 1]]
    out["count_rel_diff_at_densify"] = {str(i + 1): float(abs(ca[i] - cb[i]) / cb[i]) for i in dens}
    out["mean_rel_loss_diff_last_500"] = float(np.mean(np.abs(la[-500:] - lb[-500:]) / lb[-500:]))
    out["test_psnr_diff"] = a["test_psnr"] - b["test_psnr"]
    out["counts_equal_every_iteration"] = bool(np.array_equal(ca, cb))
    out["final_state_bitwise_equal"] = {k: bool(torch.equal(states[0][k], states[1][k])) if states[0][k] is not None
                                        else None for k in states[0]}
    for r in out["routes"].values():    # keep the record small: losses every 10 iterations
        r["losses"] = r["losses"][::10]
        r["counts"] = r["counts"][::10]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/t30k/run.json")
    ap.add_argument("--iterations", type=int, default=0, help="override trainer.max_iterations (0: the YAML's)")
    ap.add_argument("--every", type=int, default=1000)
    ap.add_argument("--compare", type=int, default=0)
    ap.add_argument("--n-true", type=int, default=1_000_000)
    ap.add_argument("--n-init", type=int, default=100_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--fx", type=float, default=1000.0)
    ap.add_argument("--views", type=int, default=24)
    ap.add_argument("--mask", choices=("yaml", "off"), default="yaml", help="off: geometry.mask false (probe only)")
    args = ap.parse_args()
    assert torch.cuda.is_available(), "needs a HIP device"
    dev = torch.device("cuda:0")
    import dogs_amd._lib as L
    L.load()
    rec = run_compare(args, dev) if args.compare else run_full(args, dev)
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(rec, f, indent=1)
    log(json.dumps({k: v for k, v in rec.items() if k not in ("trace", "routes")}))


if __name__ == "__main__":
    main()
