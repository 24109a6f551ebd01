"""Distribution of phase-1 instances per 64-Gaussian wave on the bench scene (the binning walks'
unit of work): one forward, the binned (tile, Gaussian) pairs read back, bincount per Gaussian, summed per 64.
usage: python tools/wave_inst_stats.py [N] [W] [H]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
from raster_util import hip_sorted_instances  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
W = int(sys.argv[2]) if len(sys.argv) > 2 else 1920
H = int(sys.argv[3]) if len(sys.argv) > 3 else 1080
dev = torch.device("cuda:0")
s, gc, gi = bench.make_inputs(N, W, H, 0, dev)
v = bench.View(s, gc, gi, dev)
for _ in range(3):
    out = v.forward()
torch.cuda.synchronize()
tiles, gids, e1 = hip_sorted_instances(out, W, H, dev, N)
per_g = np.bincount(gids[:e1].astype(np.int64), minlength=N)
nw = (N + 63) // 64
per_w = np.add.reduceat(np.pad(per_g, (0, nw * 64 - N)), np.arange(0, nw * 64, 64))
steps = (per_w + 63) // 64
q = lambda a, p: float(np.percentile(a, p))  # noqa: E731
print(f"E1 {e1}  Gaussians binned {int((per_g > 0).sum())}  max per Gaussian {int(per_g.max())}")
print(f"instances per wave: mean {per_w.mean():.1f} p50 {q(per_w, 50):.0f} p90 {q(per_w, 90):.0f} "
      f"p99 {q(per_w, 99):.0f} p99.9 {q(per_w, 99.9):.0f} max {int(per_w.max())}")
print(f"64-wide steps per wave: mean {steps.mean():.2f} max {int(steps.max())}  waves with >8 steps "
      f"{int((steps > 8).sum())}  >16 {int((steps > 16).sum())}")
top = np.argsort(-per_g)[:10]
print("largest Gaussians (instances):", [int(per_g[i]) for i in top])
