"""BASELINE config 2's masked iteration (bench.masked_iteration_leg's trainer) split into host and GPU time: the host
time of each train_iteration() call without a sync (median) against the synchronised wall time per iteration; run it
under rocprofv3 --kernel-trace and tools/step_gaps.py shows where the GPU idles.
python tools/masked_step_probe.py [--iters 60] [--unfold-shuffle]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--unfold-shuffle", action="store_true",
                    help="run the stages' PixelShuffle as its own torch op (the A/B of the folded one)")
    args = ap.parse_args()
    if args.unfold_shuffle:
        import torch.nn.functional as F
        from dogs_amd.masks import Conv3x3
        fold = Conv3x3.forward

        def unfolded(self, x, relu=False, shuffle=False):
            return fold(self, F.pixel_shuffle(x, 2) if shuffle else x, relu)
        Conv3x3.forward = unfolded
    import bench
    from dogs_amd.synthetic import make_scene
    dev = torch.device("cuda", 0)
    s = make_scene(1_000_000, 1920, 1080, seed=1234).to(dev)
    cams = bench.make_cameras(1920, 1080, bench.view_yaws(8), dev)
    import json
    from dataclasses import replace
    from dogs_amd.gaussian_model import GaussianSplatModel
    from dogs_amd.trainer import GaussianSplatTrainer, GSTrainConfig
    with open(os.path.join(ROOT, "tests", "golden", "reference_configs.json")) as f:
        cfg = GSTrainConfig.from_reference(json.load(f)["mipnerf360.yaml"])
    cfg = replace(cfg, densify_start_iter=10 ** 9, opacity_reset_interval=10 ** 9, spatial_lr_scale=1.0)
    m = GaussianSplatModel(3, cfg.percent_dense, dev)
    m.init_from_external_properties(s.means3D, s.dc, s.sh, s.raw_scales, s.raw_rotations, s.raw_opacities)
    m.active_sh_degree = 3
    g = torch.Generator().manual_seed(11)
    gts = [torch.rand((3, c.height, c.width), generator=g).to(dev) for c in cams]
    torch.manual_seed(0)
    tr = GaussianSplatTrainer(m, cams, gts, cfg, device=dev, seed=0, native=True)
    for _ in range(10):
        tr.train_iteration()
    tr.sync()
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for _ in range(args.iters):
        th = time.perf_counter()
        tr.train_iteration()
        host.append(time.perf_counter() - th)
    tr.sync()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.iters * 1e3
    print(f"masked iteration: wall {wall:.3f} ms, host median {np.median(host) * 1e3:.3f} ms "
          f"(p10 {np.percentile(host, 10) * 1e3:.3f}, p90 {np.percentile(host, 90) * 1e3:.3f})", flush=True)


if __name__ == "__main__":
    main()
