"""Debug helper: forward+backward of a small scene through the _C table, grads saved to an .npz (DOGS_HIP_LIB picks
the library).  usage: python tools/dbg/grads.py OUT.npz"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from raster_util import hip_forward, small_scene  # noqa: E402
from dogs_amd.diff_gaussian_rasterization import _C  # noqa: E402

dev = torch.device("cuda:0")
n, W, H = 1024, 133, 97
s = small_scene(n, W, H, seed=11 + n)
bg = (1, 1, 1)
out = hip_forward(s, bg, dev)
rng = np.random.default_rng(0)
gcol = rng.standard_normal((3, H, W)).astype(np.float32)
c = s.camera.to(dev)
e = torch.empty(0, device=dev)
d = lambda t: t.to(dev).contiguous()  # noqa: E731
gr = _C.rasterize_gaussians_backward(
    torch.as_tensor(bg, dtype=torch.float32, device=dev), d(s.means3D), out[4], e, d(s.opacities), d(s.scales),
    d(s.rotations), 1.0, e, c.world_to_camera, c.projective_matrix, c.tanfovx, c.tanfovy,
    torch.from_numpy(gcol).to(dev), d(s.dc), d(s.sh), torch.zeros((1, H, W), device=dev), 3, c.camera_center,
    out[5], out[0], out[6], out[7], out[1], out[8], False, False)
names = ["dmeans2D", "dcolors", "dopacity", "dmeans3D", "dcov3D", "ddc", "dsh", "dscales", "drot", "depth"]
np.savez(sys.argv[1], **{k: v.cpu().numpy() for k, v in zip(names, gr)})
from raster_util import hip_geometry  # noqa: E402
xy, co, rgbi, cnt = hip_geometry(out, n, dev)
np.save(sys.argv[1].replace(".npz", "_cnt.npy"), cnt)
