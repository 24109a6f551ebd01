"""Where the native route (dg_train_step) and the autograd route (render() + SparseGaussianAdam) of
GaussianSplatTrainer first differ: both run from the same state, iteration by iteration, and after each iteration
every parameter, Adam moment and densification statistic is compared bit for bit.  Prints the first differing
iteration per tensor and the size of the difference.

    python tools/route_probe.py [--mask] [--iters 10]
"""
import argparse
import copy
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mask", action="store_true")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--W", type=int, default=400)
    ap.add_argument("--H", type=int, default=300)
    ap.add_argument("--ref", action="store_true", help="tools/train_30k.py's problem and mipnerf360.yaml schedule")
    args = ap.parse_args()
    from test_gpu_trainer import _cfg, _normal, _problem
    from dogs_amd.masks import AppearanceEmbedding
    from dogs_amd.trainer import GaussianSplatTrainer
    dev = torch.device("cuda:0")
    kw = dict(densify_start_iter=10 ** 6, opacity_reset_interval=10 ** 6, prune_iterations=(), sh_increase_interval=3)
    if args.mask:
        kw.update(mask=True, lambda_mask=0.5, depth_threshold=6.0)
    cfg = _cfg(**kw)
    torch.manual_seed(1)
    net0 = AppearanceEmbedding(4)
    trs = []
    for native in (True, False):
        if args.ref:
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            import train_30k as T
            cfg = T.reference_cfg()
            m, cams, gts = T.problem(dev, 1_000_000, 100_000, 1920, 1080, 1000.0, 24)
            tr_idx, _ = T.split(cams, gts)
            torch.manual_seed(0)
            tr = GaussianSplatTrainer(m, [cams[i] for i in tr_idx], [gts[i] for i in tr_idx], cfg, device=dev,
                                      seed=42, native=native, normal=_normal(dev, 7))
        else:
            m, cams, gts = _problem(dev, n_true=30_000, n_init=6_000, W=args.W, H=args.H, views=4)
            tr = GaussianSplatTrainer(m, cams, gts, cfg, device=dev, seed=2, native=native, normal=_normal(dev, 3),
                                      appear_embedding=copy.deepcopy(net0) if args.mask else None)
        trs.append(tr)
    first = {}
    for it in range(1, args.iters + 1):
        snaps = []
        for tr in trs:
            tr.train_iteration()
            tr.sync()
            m = tr.model
            opt = {g["name"]: tr.optimizer.state[g["params"][0]] for g in tr.optimizer.param_groups}
            d = {f"param.{k}": v.detach().clone() for k, v in m.params().items()}
            d.update({f"m.{k}": v["exp_avg"].clone() for k, v in opt.items()})
            d.update({f"v.{k}": v["exp_avg_sq"].clone() for k, v in opt.items()})
            d.update({"grad_accum": m.xyz_gradient_accum.clone(), "denom": m.denom.clone(),
                      "max_radii2D": m.max_radii2D.clone()})
            if tr.mask is not None:
                d.update({f"net.{k}": v.detach().clone() for k, v in tr.mask.state_dict().items()})
            snaps.append(d)
        a, b = snaps
        for k in a:
            if k not in first and not torch.equal(a[k], b[k]):
                diff = float((a[k].double() - b[k].double()).abs().max())
                nd = int((a[k] != b[k]).sum())
                first[k] = (it, diff, nd)
                print(f"iteration {it}: {k} differs (max |d| {diff:.3e}, {nd} elements)", flush=True)
        print(f"iteration {it}: {sum(1 for k in a if not torch.equal(a[k], b[k]))} of {len(a)} tensors differ",
              flush=True)


if __name__ == "__main__":
    main()
