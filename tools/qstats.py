"""Reads the DG_QSTATS counters of one forward of the bench scene (build: tools/build_variant.sh ab/qstats.so
-DDG_QSTATS; run with DOGS_HIP_LIB=ab/qstats.so): splats per processed batch for the tile vs its busiest quadrant."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dogs_amd.synthetic import make_scene  # noqa: E402

dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
s = make_scene(n, 1920, 1080, seed=1234).to(dev)
v = bench.View(s, torch.randn((3, 1080, 1920), device=dev), torch.zeros((1, 1080, 1920), device=dev), dev) \
    if hasattr(bench, "View") else None
out = v.forward()
torch.cuda.synchronize()
c = out[5][:64].view(torch.int32).cpu().tolist()
print(f"c13 {c[13]} c14 {c[14]} c15 {c[15]} ratio14 {c[14] / max(c[13], 1):.3f}")
