"""SparseGaussianAdam.step over the six groups of 1e6 Gaussians (59 floats each, 88% visible): one launch
(dg_adam_update_groups); reports us/step and the effective HBM rate of 28 B per visible float.
usage: python tools/adam_bench.py [N] (DOGS_HIP_LIB selects a library variant)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diff_gaussian_rasterization import SparseGaussianAdam  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
dev = torch.device("cuda:0")
shapes = {"xyz": (3,), "f_dc": (1, 3), "f_rest": (15, 3), "opacity": (1,), "scaling": (3,), "quaternion": (4,)}
ps = {k: torch.nn.Parameter(torch.randn((N,) + s, device=dev)) for k, s in shapes.items()}
opt = SparseGaussianAdam([{"params": [p], "lr": 1e-3, "name": k} for k, p in ps.items()], lr=0.0, eps=1e-15)
for p in ps.values():
    p.grad = torch.randn_like(p)
vis = torch.rand(N, device=dev) < 0.88
for _ in range(3):
    opt.step(vis, N)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
e0.record()
for _ in range(20):
    opt.step(vis, N)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / 20 * 1e3
nbytes = 28 * 59 * float(vis.sum())
print(f"{os.environ.get('DOGS_HIP_LIB', 'default')}: {us:.1f} us/step, {nbytes / us / 1e3:.0f} GB/s effective")
