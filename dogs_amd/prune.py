"""LightGaussian pruning (conerf/model/gaussian_fields/prune.py:14-65, conerf/render/gaussian_render.py:161-278).

* `count_render(model, camera, pipeline_config, bkgd_color)` -- the count-mode forward (dg_rasterize_count: per
  Gaussian, the pixels it contributes to and opacity x that count), with the reference's result dict.  The reference's
  own call cannot run (its settings omit `antialiasing` and pass `f_count`, which its binding lacks);
  this one accepts exactly those settings.
* `prune_list(model, cameras, ...)` -- sums of the counts and scores over the cameras (:35-65), accumulated on the
  device in camera order as the reference does (`cameras.pop()`: last camera first).
* `calculate_v_imp_score(model, imp_list, v_pow)` -- (:14-32) volume-weighted importance.

With the model's prune_gaussians_with_opt (dogs_amd.gaussian_model) this is the whole device-side prune step of the
trainer (gaussian_trainer.py:457-470) and of the ADMM phase entry (master_gaussian_trainer.py:103-121): count renders,
one sort for the percentile, one compaction of the parameters and their Adam moments."""
from __future__ import annotations

import math

import torch

from .diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer


def _tan_half(cam, axis: str) -> float:
    t = getattr(cam, "tanfov" + axis, None)
    return float(t) if t is not None else math.tan(getattr(cam, "fov_" + axis) * 0.5)


@torch.no_grad()
def count_render(gaussian_splat_model, viewpoint_camera, pipeline_config, bkgd_color: torch.Tensor,
                 scaling_modifier: float = 1.0, anti_aliasing: bool = False, override_color=None,
                 subpixel_offset=None, device="cuda:0") -> dict:
    """gaussian_render.py:161-278."""
    m, cam = gaussian_splat_model, viewpoint_camera
    settings = GaussianRasterizationSettings(
        image_height=int(cam.height), image_width=int(cam.width), tanfovx=_tan_half(cam, "x"),
        tanfovy=_tan_half(cam, "y"), bg=bkgd_color, scale_modifier=scaling_modifier,
        viewmatrix=cam.world_to_camera, projmatrix=cam.projective_matrix, sh_degree=m.active_sh_degree,
        campos=cam.camera_center, prefiltered=False, debug=bool(getattr(pipeline_config, "debug", False)),
        antialiasing=anti_aliasing, depth_threshold=0.0, f_count=True)
    rast = GaussianRasterizer(raster_settings=settings)
    scales = rotations = cov3D = None
    if getattr(pipeline_config, "compute_cov3D_python", False):
        cov3D = m.get_covariance(scaling_modifier)
    else:
        rotations, scales = m.get_quaternion, m.get_scaling
    colors = override_color
    shs = m.get_features if override_color is None else None
    count, score, image, radii = rast(means3D=m.get_xyz.detach(), means2D=None, opacities=m.get_opacity.detach(),
                                      shs=shs.detach() if shs is not None else None, colors_precomp=colors,
                                      scales=scales.detach() if scales is not None else None,
                                      rotations=rotations.detach() if rotations is not None else None,
                                      cov3D_precomp=cov3D)
    return {"rendered_image": image, "visibility_filter": radii > 0, "radii": radii, "gaussians_count": count,
            "important_score": score}


@torch.no_grad()
def prune_list(gaussians, cameras: list, pipeline_config=None, bkgd_color: torch.Tensor | None = None):
    """prune.py:35-65: (gaussians_count, important_score) summed over the cameras, taken from the end of the list as
    the reference's cameras.pop() does (the caller's list is not modified)."""
    dev = gaussians.get_xyz.device
    if bkgd_color is None:
        bkgd_color = torch.zeros(3, dtype=torch.float32, device=dev)
    count = imp = None
    for cam in reversed(list(cameras)):
        cam = cam.to(dev) if hasattr(cam, "to") else cam
        r = count_render(gaussians, cam, pipeline_config, bkgd_color)
        if count is None:
            count, imp = r["gaussians_count"], r["important_score"]
        else:
            count += r["gaussians_count"]
            imp += r["important_score"]
    return count, imp


@torch.no_grad()
def calculate_v_imp_score(gaussians, imp_list: torch.Tensor, v_pow: float) -> torch.Tensor:
    """prune.py:14-32: (volume / 90th-percentile-from-the-top volume) ** v_pow x importance."""
    volume = torch.prod(gaussians.get_scaling, dim=1)
    index = int(len(volume) * 0.9)
    sorted_volume, _ = torch.sort(volume, descending=True)
    kth_percent_largest = sorted_volume[index]
    v_list = torch.pow(volume / kth_percent_largest, v_pow)
    return v_list * imp_list
