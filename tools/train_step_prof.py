"""Runs bench.TrainStep alone (N=1e6, 1080p) for a kernel trace of the training iteration:
rocprofv3 --kernel-trace --stats -d OUT -- python tools/train_step_prof.py [steps]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dogs_amd.synthetic import make_scene  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda:0")
s = make_scene(1_000_000, 1920, 1080, seed=1234).to(dev)
ts = bench.TrainStep(s, dev, 1234)
for _ in range(3):
    ts.step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    ts.step()
torch.cuda.synchronize()
print(f"train step {(time.perf_counter() - t0) / steps * 1e3:.3f} ms")
print(f"densify_and_prune {ts.densify()}")
