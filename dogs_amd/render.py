"""`render()` -- the entry of the hot path, drop-in for conerf/render/gaussian_render.py:18-158.

Same arguments, same result dict (rendered_image, screen_space_points, visibility_filter, radii, scaling, depth).
The model and camera are duck-typed as in the reference: the model exposes get_xyz, get_opacity, get_scaling,
get_quaternion, get_features / get_features_dc / get_features_rest, active_sh_degree, max_sh_degree,
get_covariance(scaling_modifier) and get_exposure_from_id(index); the camera fov_x, fov_y, width, height,
world_to_camera, projective_matrix, camera_center (and image_index for the exposure); the pipeline config debug,
compute_cov3D_python, convert_SHs_python.  Everything runs on the device through this package's rasterizer
(libdogs_hip); the optional Python-side SH evaluation (convert_SHs_python) is the reference's torch expression
(sh_utils.py:57-112) evaluated with the coefficient table below.
"""
from __future__ import annotations

import math

import torch

from .diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer

# real SH basis constants by band (sh_utils.py:17-49), degree <= 3 (the rasterizer's limit)
_SH_C0 = 0.28209479177387814
_SH_C1 = 0.4886025119029199
_SH_C2 = (1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396)
_SH_C3 = (-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
          1.445305721320277, -0.5900435899266435)


def eval_sh(deg: int, sh: torch.Tensor, dirs: torch.Tensor) -> torch.Tensor:
    """sh [..., C, (deg+1)^2] at unit directions [..., 3] -> [..., C]; the reference's term order (sh_utils.py:57)."""
    if not 0 <= deg <= 3:
        raise ValueError(f"SH degree {deg} unsupported (0..3)")
    if sh.shape[-1] < (deg + 1) ** 2:
        raise ValueError("too few SH coefficients for the degree")
    out = _SH_C0 * sh[..., 0]
    if deg == 0:
        return out
    x, y, z = dirs[..., 0:1], dirs[..., 1:2], dirs[..., 2:3]
    out = out - _SH_C1 * y * sh[..., 1] + _SH_C1 * z * sh[..., 2] - _SH_C1 * x * sh[..., 3]
    if deg == 1:
        return out
    xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
    # each term is ((c * f0) * f1 ...) * sh[k]: the reference's left-to-right products, so the values match bitwise
    bands = [((xy,), (yz,), (2.0 * zz - xx - yy,), (xz,), (xx - yy,))]
    if deg > 2:
        bands.append(((y, 3 * xx - yy), (xy, z), (y, 4 * zz - xx - yy), (z, 2 * zz - 3 * xx - 3 * yy),
                      (x, 4 * zz - xx - yy), (z, xx - yy), (x, xx - 3 * yy)))
    k = 4
    for consts, factors in zip((_SH_C2, _SH_C3), bands):
        for c, fs in zip(consts, factors):
            t = c * fs[0]
            for f in fs[1:]:
                t = t * f
            out = out + t * sh[..., k]
            k += 1
    return out


def render(gaussian_splat_model, viewpoint_camera, pipeline_config, bkgd_color: torch.Tensor,
           scaling_modifier: float = 1.0, anti_aliasing: bool = False, override_color: torch.Tensor | None = None,
           separate_sh: bool = False, use_trained_exposure: bool = False, depth_threshold: float = 0.0,
           device="cuda:0") -> dict:
    m = gaussian_splat_model
    cam = viewpoint_camera
    xyz = m.get_xyz
    # zeros + 0: a non-leaf tensor whose .grad autograd fills (retain_grad), the reference's means2D carrier
    screen_space_points = torch.zeros_like(xyz, dtype=xyz.dtype, requires_grad=True, device=device) + 0
    try:
        screen_space_points.retain_grad()
    except RuntimeError:
        pass
    settings = GaussianRasterizationSettings(
        image_height=int(cam.height), image_width=int(cam.width),
        tanfovx=math.tan(cam.fov_x * 0.5), tanfovy=math.tan(cam.fov_y * 0.5),
        bg=bkgd_color, scale_modifier=scaling_modifier, viewmatrix=cam.world_to_camera,
        projmatrix=cam.projective_matrix, sh_degree=m.active_sh_degree, campos=cam.camera_center,
        prefiltered=False, debug=bool(getattr(pipeline_config, "debug", False)), antialiasing=anti_aliasing,
        depth_threshold=depth_threshold)
    rasterizer = GaussianRasterizer(raster_settings=settings)

    scales = rotations = cov3D_precomp = None
    if getattr(pipeline_config, "compute_cov3D_python", False):
        cov3D_precomp = m.get_covariance(scaling_modifier)
    else:
        rotations = m.get_quaternion
        scales = m.get_scaling

    shs = colors_precomp = dc = None
    if override_color is not None:
        colors_precomp = override_color
    elif getattr(pipeline_config, "convert_SHs_python", False):
        feats = m.get_features
        shs_view = feats.transpose(1, 2).view(-1, 3, (m.max_sh_degree + 1) ** 2)
        dir_pp = xyz - cam.camera_center.repeat(feats.shape[0], 1)
        dir_pp = dir_pp / dir_pp.norm(dim=1, keepdim=True)
        colors_precomp = torch.clamp_min(eval_sh(m.active_sh_degree, shs_view, dir_pp) + 0.5, 0.0)
    elif separate_sh:
        dc, shs = m.get_features_dc, m.get_features_rest
    else:
        shs = m.get_features

    kw = dict(means3D=xyz, means2D=screen_space_points, shs=shs, colors_precomp=colors_precomp,
              opacities=m.get_opacity, scales=scales, rotations=rotations, cov3D_precomp=cov3D_precomp)
    if separate_sh:
        kw["dc"] = dc
    image, radii, depth = rasterizer(**kw)

    if use_trained_exposure:
        exposure = m.get_exposure_from_id(cam.image_index)
        image = torch.matmul(image.permute(1, 2, 0), exposure[:3, :3]).permute(2, 0, 1) + exposure[:3, 3, None, None]
    image = image.clamp(0, 1)
    return {"rendered_image": image, "screen_space_points": screen_space_points, "visibility_filter": radii > 0,
            "radii": radii, "scaling": scales, "depth": depth}
