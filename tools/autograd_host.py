"""Host time per phase of the autograd-route train step (bench.TrainStep.step: the drop-in calls as the reference
trainer makes them), without a profiler: perf_counter stamps between the phases of one step, medians over --steps.
The forward's stamp includes its wait for the phase-1 counters (the GPU catches up there); everything after it is
pure enqueue time while the GPU works through the render -- when that exceeds the GPU work queued, the GPU idles.
python tools/autograd_host.py [--steps 60]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--n", type=int, default=1_000_000)
    args = ap.parse_args()
    import bench
    from dogs_amd.synthetic import make_scene
    dev = torch.device("cuda", 0)
    W, H = 1920, 1080
    s = make_scene(args.n, W, H, seed=1234).to(dev)
    cams = bench.make_cameras(W, H, bench.view_yaws(8), dev)
    ts = bench.TrainStep(s, cams, dev, 1234)
    marks = {}

    def step():
        t = [time.perf_counter()]
        p = ts.params
        rast = ts.rasts[ts.i % len(ts.rasts)]
        ts.i += 1
        m2d = torch.zeros_like(p["xyz"], requires_grad=True)
        opac, scales, rots = ts.activate(p["opacity"], p["scaling"], p["quaternion"])
        t.append(time.perf_counter())
        img, radii, _ = rast(means3D=p["xyz"], means2D=m2d, opacities=opac, dc=p["f_dc"], shs=p["f_rest"],
                             scales=scales, rotations=rots)
        t.append(time.perf_counter())
        img, l1 = ts.clamp_l1(img, ts.gt)
        ssim = ts.fused_ssim(img.unsqueeze(0), ts.gt.unsqueeze(0))
        t.append(time.perf_counter())
        loss = 0.8 * l1 + 0.2 * (1.0 - ssim) + 0.05 * ts.row_prod(scales).mean()
        t.append(time.perf_counter())
        loss.backward()
        t.append(time.perf_counter())
        vis = radii > 0
        ts.opt.step(vis, radii.shape[0], stats=dict(ts.stats, radii=radii, dmeans2D=m2d.grad))
        t.append(time.perf_counter())
        ts.opt.zero_grad(set_to_none=True)
        t.append(time.perf_counter())
        for k, name in enumerate(("activate", "raster_forward(+wait)", "clamp_l1+ssim", "loss_expr", "backward",
                                  "adam_step", "zero_grad")):
            marks.setdefault(name, []).append(1e6 * (t[k + 1] - t[k]))
        marks.setdefault("total", []).append(1e6 * (t[-1] - t[0]))

    for _ in range(16):
        step()
    torch.cuda.synchronize()
    marks.clear()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.steps * 1e6
    print(f"autograd route: {wall:.1f} us per step (wall, {args.steps} steps)")
    for k, v in marks.items():
        print(f"  {k:24s} host median {np.median(v):8.1f} us  min {np.min(v):8.1f}")


if __name__ == "__main__":
    main()
