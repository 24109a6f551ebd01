"""Grid2D block split timing: dogs_amd.blocksplit (GPU passes) vs the CPU restatement (numpy, one pass per box, as
the reference), on a synthetic COLMAP-like cloud.  usage: python tools/blocksplit_bench.py [N] [MX] [MY]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dogs_amd import blocksplit as G  # noqa: E402
from oracle import blocksplit_oracle as O  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
MX = int(sys.argv[2]) if len(sys.argv) > 2 else 4
MY = int(sys.argv[3]) if len(sys.argv) > 3 else 4
rng = np.random.default_rng(0)
pts = np.concatenate([rng.normal(size=(N, 2)) * [400.0, 150.0], rng.normal(size=(N, 1))], axis=1)
dev = torch.device("cuda:0")
pd = torch.from_numpy(pts).to(dev)
T, _ = O.oriented_bounds_2D(pts[:100_000, :2])


def split_gpu():
    lab, cells, exp, _ = G.Grid2DClustering(pd, mx=MX, my=MY, p0=0.00001, p1=0.99999, transform_world_to_obb=T)
    mem = G.points_in_boxes2d(pd, [e[:, :2] for e in exp], T, device=dev)["members"]
    torch.cuda.synchronize()
    return lab, mem


split_gpu()
t0 = time.perf_counter()
R = 5
for _ in range(R):
    lab, mem = split_gpu()
gpu_s = (time.perf_counter() - t0) / R
# one fused pass alone (the kernel's streaming rate): labels + members of MX*MY boxes
boxes = [np.array([[-1e3 + 100 * k, -300.0], [-1e3 + 100 * k + 400, 300.0]]) for k in range(MX * MY)]
G.points_in_boxes2d(pd, boxes, T, labels=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(R):
    G.points_in_boxes2d(pd, boxes, T, labels=True)
torch.cuda.synchronize()
pass_s = (time.perf_counter() - t0) / R
t0 = time.perf_counter()
lab_o, cells_o, exp_o, _ = O.Grid2DClustering(pts, mx=MX, my=MY, p0=0.00001, p1=0.99999, transform_world_to_obb=T)
mem_o = [O.points_in_bbox2D(pts, e, T) for e in exp_o]
cpu_s = time.perf_counter() - t0
assert np.array_equal(lab, lab_o)
assert all(np.array_equal(a.cpu().numpy(), b) for a, b in zip(mem, mem_o))
print(f"blocksplit N={N} {MX}x{MY}: GPU split {gpu_s * 1e3:.1f} ms (one fused box pass {pass_s * 1e3:.2f} ms, "
      f"{N * 16 / pass_s / 1e9:.0f} GB/s of point reads), CPU restatement {cpu_s * 1e3:.0f} ms; identical output")
