"""Export timing: save_splat / save_ply of N Gaussians through dogs_amd.export (GPU pack +
one host write) against the reference's per-Gaussian Python loop (oracle/export_oracle.splat_body, the same loop)
timed on a sample and scaled.  usage: python tools/export_bench.py [N] [sample]"""
import os
import sys
import tempfile
import time
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dogs_amd import export  # noqa: E402
from oracle import export_oracle as X  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
sample = int(sys.argv[2]) if len(sys.argv) > 2 else 20_000
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
m = types.SimpleNamespace(_xyz=torch.randn((n, 3), generator=g).to(dev),
                          _features_dc=torch.randn((n, 1, 3), generator=g).to(dev),
                          _scaling=(torch.randn((n, 3), generator=g) - 4).to(dev),
                          _opacity=torch.randn((n, 1), generator=g).to(dev),
                          _quaternion=torch.randn((n, 4), generator=g).to(dev))
d = tempfile.mkdtemp()
res = {}
for name, fn in (("save_splat", export.save_splat), ("save_ply", export.save_ply)):
    fn(m, os.path.join(d, "w"))  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn(m, os.path.join(d, "x"))
    torch.cuda.synchronize()
    res[name] = time.perf_counter() - t0
a = [getattr(m, k)[:sample].cpu().numpy() for k in ("_xyz", "_scaling", "_opacity", "_quaternion", "_features_dc")]
t0 = time.perf_counter()
X.splat_body(*a)
ref = (time.perf_counter() - t0) / sample * n
print(f"N={n}: save_splat {res['save_splat'] * 1e3:.1f} ms, save_ply {res['save_ply'] * 1e3:.1f} ms (GPU pack + write); "
      f"reference per-Gaussian save_splat loop ~{ref:.1f} s on 1 core (timed on {sample}, scaled)")
