"""Generate the golden fixtures under tests/golden/ (run in the build container, never on the GPU box).

    python tests/golden/make_golden.py

Inputs are small seeded scenes from dogs_amd.synthetic (BASELINE.md §2 generator).  Expected outputs come from
the REFERENCE's own Python where it has the arithmetic, imported by file path from
/root/reference -- nothing from the reference is copied into the repository, only these vectors:

  golden_sh_cov.npz   precomputed colours of the reference's python SH path
                      (conerf/render/gaussian_render.py:87-102 -> sh_utils.eval_sh :57, clamp_min(+0.5, 0))
                      for SH degree 0..3, and the 3D covariance L L^T with L from
                      utils.rotation_mat_left_multiply_scale_mat :70 (gaussian_splat_model.py:111-117; the six
                      entries taken as (00, 01, 02, 11, 12, 22) -- the reference's strip_symmetric writes
                      Sigma[2,1] into slot 5, utils.py:14, which the CUDA path does not do)
  golden_ssim.npz     conerf/loss/ssim_torch.ssim :82 value and its autograd gradient w.r.t. img1
                      (same 11-tap sigma-1.5 window and zero padding as fused-ssim's "same" mode)
  golden_raster_*.npz frozen outputs of the CPU oracle (oracle/gs_oracle.c) for small scenes: image,
                      inverse depth, radii, num_rendered, the sorted (tile, Gaussian) list and all ten
                      backward outputs -- regression vectors for the oracle itself (no reference binary
                      exists for the CUDA rasterizer: SURVEY.md §8(c)).
"""
from __future__ import annotations

import importlib.util
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/conerf"
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def scene_arrays(n, W, H, seed):
    from raster_util import small_scene
    s = small_scene(n, W, H, seed=seed)
    c = s.camera
    return dict(means3D=s.means3D.numpy(), scales=s.scales.numpy(), rotations=s.rotations.numpy(),
                opacities=s.opacities.numpy(), dc=s.dc.numpy(), sh=s.sh.numpy(),
                viewmatrix=c.world_to_camera.numpy(), projmatrix=c.projective_matrix.numpy(),
                campos=c.camera_center.numpy(), tanfovx=np.float32(c.tanfovx), tanfovy=np.float32(c.tanfovy),
                W=np.int32(W), H=np.int32(H))


def make_sh_cov(out):
    sh_utils = _load("ref_sh_utils", f"{REF}/model/gaussian_fields/sh_utils.py")
    gutils = _load("ref_gs_utils", f"{REF}/model/gaussian_fields/utils.py")
    a = scene_arrays(256, 133, 97, seed=3)
    means = torch.from_numpy(a["means3D"])
    feats = torch.cat([torch.from_numpy(a["dc"]), torch.from_numpy(a["sh"])], dim=1)  # [N,16,3]
    shs_view = feats.transpose(1, 2).reshape(-1, 3, 16)
    dir_pp = means - torch.from_numpy(a["campos"]).reshape(1, 3).repeat(means.shape[0], 1)
    dirn = dir_pp / dir_pp.norm(dim=1, keepdim=True)
    for deg in range(4):
        a[f"rgb_deg{deg}"] = torch.clamp_min(sh_utils.eval_sh(deg, shs_view, dirn) + 0.5, 0.0).numpy()
    L = gutils.rotation_mat_left_multiply_scale_mat(torch.from_numpy(a["scales"]), torch.from_numpy(a["rotations"]))
    S = L @ L.transpose(1, 2)
    a["cov3D"] = torch.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1], S[:, 1, 2], S[:, 2, 2]], 1).numpy()
    np.savez_compressed(os.path.join(out, "golden_sh_cov.npz"), **a)


def make_ssim(out):
    ssim_torch = _load("ref_ssim_torch", f"{REF}/loss/ssim_torch.py")
    g = torch.Generator().manual_seed(5)
    res = {}
    for tag, (H, W) in (("a", (37, 53)), ("b", (64, 64))):
        img1 = torch.rand((1, 3, H, W), generator=g)
        img2 = (img1 + 0.1 * torch.randn((1, 3, H, W), generator=g)).clamp(0, 1)
        x = img1.clone().requires_grad_(True)
        val = ssim_torch.ssim(x, img2)
        val.backward()
        res[f"{tag}_img1"] = img1.numpy()
        res[f"{tag}_img2"] = img2.numpy()
        res[f"{tag}_value"] = np.float32(val.item())
        res[f"{tag}_grad"] = x.grad.numpy()
    np.savez_compressed(os.path.join(out, "golden_ssim.npz"), **res)


RASTER_CASES = {
    # name: (n, W, H, deg, bg, antialiasing)
    "golden_raster_64x48.npz": (64, 64, 48, 3, (0.1, 0.5, 0.9), False),
    "golden_raster_133x97_aa.npz": (300, 133, 97, 1, (0.0, 0.0, 0.0), True),
}


def make_raster(out):
    from oracle import oracle as O
    O.build()
    for name, (n, W, H, deg, bg, aa) in RASTER_CASES.items():
        a = scene_arrays(n, W, H, seed=21 + n)
        col, radii, invd, st = O.forward(a["means3D"], a["opacities"], a["viewmatrix"], a["projmatrix"], a["campos"],
                                         float(a["tanfovx"]), float(a["tanfovy"]), H, W, np.asarray(bg, np.float32),
                                         dc=a["dc"], sh=a["sh"], scales=a["scales"], rotations=a["rotations"],
                                         sh_degree=deg, antialiasing=aa)
        rng = np.random.default_rng(n)
        gcol = rng.standard_normal((3, H, W)).astype(np.float32)
        ginv = (0.1 * rng.standard_normal((H, W))).astype(np.float32)
        go = st.backward(gcol, ginv)
        tiles, gids, _ = st.sorted_list()
        res = dict(a, bg=np.asarray(bg, np.float32), deg=np.int32(deg), antialiasing=np.int32(aa),
                   color=col, invdepth=invd, radii=radii, num_rendered=np.int64(st.num_rendered),
                   num_instances=np.int64(st.num_valid), tiles=tiles, gids=gids, ranges=st.ranges(),
                   grad_color=gcol, grad_invdepth=ginv)
        for k, v in go.items():
            res["g_" + k] = v
        np.savez_compressed(os.path.join(out, name), **res)


if __name__ == "__main__":
    make_sh_cov(HERE)
    make_ssim(HERE)
    make_raster(HERE)
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)), "bytes")
