"""Times fused-SSIM forward (train) + backward at 1080p x 3 channels: python tools/ssim_bench.py [iters]
(DOGS_HIP_LIB selects a library variant)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fused_ssim_cuda import fusedssim, fusedssim_backward  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
a = torch.rand((1, 3, 1080, 1920), generator=g).to(dev)
b = torch.rand((1, 3, 1080, 1920), generator=g).to(dev)
dl = torch.full_like(a, 1.0 / a.numel())
C1, C2 = 0.01 ** 2, 0.03 ** 2
for _ in range(5):
    m, d1, d2, d3 = fusedssim(C1, C2, a, b, True)
    fusedssim_backward(C1, C2, a, b, dl, d1, d2, d3)
e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
torch.cuda.synchronize()
e0.record()
for _ in range(it):
    m, d1, d2, d3 = fusedssim(C1, C2, a, b, True)
e1.record()
for _ in range(it):
    fusedssim_backward(C1, C2, a, b, dl, d1, d2, d3)
e2.record()
torch.cuda.synchronize()
print(f"{os.environ.get('DOGS_HIP_LIB', 'default')}: fwd {e0.elapsed_time(e1) / it * 1e3:.1f} us  "
      f"bwd {e1.elapsed_time(e2) / it * 1e3:.1f} us")
