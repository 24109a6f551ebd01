"""Drop-in `diff_gaussian_rasterization` for MI355X.

Mirrors the Python surface of the reference binding
(submodules/diff-gaussian-rasterization/diff_gaussian_rasterization/__init__.py):
  GaussianRasterizationSettings (:203-217), GaussianRasterizer (:220-300) with markVisible /
  visible_filter, rasterize_gaussians / _RasterizeGaussians (:25-200, incl. the depth_threshold
  scaling of grad_means2D at :171-185) and SparseGaussianAdam (:303-332).
The numerical work runs in libdogs_hip.so (gfx950 HIP kernels) through the `_C` table.
"""
from __future__ import annotations

import threading
from typing import NamedTuple

import torch
import torch.nn as nn

from . import _C

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "SparseGaussianAdam", "rasterize_gaussians", "_C"]


def cpu_deep_copy_tuple(input_tuple):
    return tuple(item.cpu().clone() if isinstance(item, torch.Tensor) else item for item in input_tuple)


# whether the caller's grad mode was on at apply time (inside Function.forward grad mode is always off, and
# ctx.needs_input_grad reports requires_grad even under torch.no_grad): only then is the backward prepared
_GRAD_MODE = threading.local()


def rasterize_gaussians(means3D, means2D, dc, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings):
    _GRAD_MODE.on = torch.is_grad_enabled()
    return _RasterizeGaussians.apply(means3D, means2D, dc, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings)


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, dc, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings):
        rs = raster_settings
        args = (rs.bg, means3D, colors_precomp, opacities, scales, rotations, rs.scale_modifier, cov3Ds_precomp,
                rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, rs.image_height, rs.image_width, dc, sh,
                rs.sh_degree, rs.campos, rs.prefiltered, rs.antialiasing, rs.debug)
        if rs.debug:
            cpu_args = cpu_deep_copy_tuple(args)
            try:
                out = _C.rasterize_gaussians(*args)
            except Exception as ex:
                torch.save(cpu_args, "snapshot_fw.dump")
                print("\nAn error occured in forward. Please forward snapshot_fw.dump for debugging.")
                raise ex
        else:
            out = _C.rasterize_gaussians(*args)
        num_rendered, num_buckets, color, invdepths, radii, geomBuffer, binningBuffer, imgBuffer, sampleBuffer = out
        # the backward's arguments (and, when no other plan holds its buffers, its outputs and scratch), prepared now:
        # the GPU is still rendering this view, so this host work is hidden here and off the backward's launch path
        ctx.plan = None
        if not rs.debug and getattr(_GRAD_MODE, "on", True) and any(ctx.needs_input_grad):
            ctx.plan = _C.backward_plan(rs.bg, means3D, colors_precomp, opacities, scales, rotations, rs.scale_modifier,
                                        cov3Ds_precomp, rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy,
                                        rs.image_height, rs.image_width, dc, sh, rs.sh_degree, rs.campos,
                                        rs.antialiasing, rs.debug, num_rendered)
        ctx.raster_settings = rs
        ctx.num_rendered = num_rendered
        ctx.num_buckets = num_buckets
        ctx.save_for_backward(colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, dc, sh, opacities,
                              geomBuffer, binningBuffer, imgBuffer, sampleBuffer)
        ctx.mark_non_differentiable(radii)
        # an unused output's gradient arrives as None instead of a zero-filled tensor (the inverse depth is usually
        # unused: a 1 x H x W fill, and another for radii, per backward); None is passed to the library as NULL
        ctx.set_materialize_grads(False)
        return color, radii, invdepths

    @staticmethod
    def backward(ctx, grad_out_color, _, grad_out_depth):
        rs = ctx.raster_settings
        (colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, dc, sh, opacities, geomBuffer,
         binningBuffer, imgBuffer, sampleBuffer) = ctx.saved_tensors
        if grad_out_color is None:
            grad_out_color = torch.zeros((3, rs.image_height, rs.image_width), dtype=torch.float32,
                                         device=means3D.device)
        if ctx.plan is not None:
            g = _C.rasterize_gaussians_backward_planned(ctx.plan, radii, grad_out_color, grad_out_depth, geomBuffer,
                                                        ctx.num_rendered, binningBuffer, imgBuffer, ctx.num_buckets,
                                                        sampleBuffer)
            ctx.plan = None
        else:
            args = (rs.bg, means3D, radii, colors_precomp, opacities, scales, rotations, rs.scale_modifier,
                    cov3Ds_precomp, rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, grad_out_color, dc, sh,
                    grad_out_depth, rs.sh_degree, rs.campos, geomBuffer, ctx.num_rendered, binningBuffer, imgBuffer,
                    ctx.num_buckets, sampleBuffer, rs.antialiasing, rs.debug)
            if rs.debug:
                cpu_args = cpu_deep_copy_tuple(args)
                try:
                    g = _C.rasterize_gaussians_backward(*args)
                except Exception as ex:
                    torch.save(cpu_args, "snapshot_bw.dump")
                    print("\nAn error occured in backward. Writing snapshot_bw.dump for debugging.\n")
                    raise ex
            else:
                g = _C.rasterize_gaussians_backward(*args)
        (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp, grad_dc, grad_sh,
         grad_scales, grad_rotations, depth) = g

        depth_threshold = getattr(rs, "depth_threshold", 0.0) or 0.0
        if depth_threshold > 0:
            scaling = torch.minimum(torch.ones_like(depth), (depth / depth_threshold) ** 2)
            grad_means2D = grad_means2D * scaling.expand_as(grad_means2D)

        return (grad_means3D, grad_means2D, grad_dc, grad_sh, grad_colors_precomp, grad_opacities, grad_scales,
                grad_rotations, grad_cov3Ds_precomp, None)


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool
    antialiasing: bool = False
    depth_threshold: float = 0.0
    # LightGaussian count mode (old_diff-gaussian-rasterization __init__.py:284-298 `f_count`, used by
    # conerf/render/gaussian_render.py:161-278 count_render): the rasterizer returns per-Gaussian contribution
    # counts and importance scores instead of a differentiable image
    f_count: bool = False


def _empty_like_device(ref: torch.Tensor) -> torch.Tensor:
    return torch.empty(0, dtype=torch.float32, device=ref.device)


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):  # noqa: N802
        with torch.no_grad():
            rs = self.raster_settings
            return _C.mark_visible(positions, rs.viewmatrix, rs.projmatrix)

    def forward(self, means3D, means2D, opacities, dc=None, shs=None, colors_precomp=None, scales=None,
                rotations=None, cov3D_precomp=None):
        rs = self.raster_settings
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception("Please provide excatly one of either SHs or precomputed colors!")
        if ((scales is None or rotations is None) and cov3D_precomp is None) or (
                (scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!")
        if getattr(rs, "f_count", False):
            return self._forward_count(means3D, opacities, dc, shs, colors_precomp, scales, rotations, cov3D_precomp)
        # extension: full SH features [N,(D+1)^2,3] without a separate dc (the reference requires dc)
        if shs is not None and (dc is None or dc.numel() == 0) and shs.dim() == 3 and shs.size(1) >= 1:
            dc, shs = shs[:, :1, :], shs[:, 1:, :]
        e = _empty_like_device(means3D)
        dc = e if dc is None else dc
        shs = e if shs is None else shs
        colors_precomp = e if colors_precomp is None else colors_precomp
        scales = e if scales is None else scales
        rotations = e if rotations is None else rotations
        cov3D_precomp = e if cov3D_precomp is None else cov3D_precomp
        return rasterize_gaussians(means3D, means2D, dc, shs, colors_precomp, opacities, scales, rotations,
                                   cov3D_precomp, rs)

    @torch.no_grad()
    def _forward_count(self, means3D, opacities, dc, shs, colors_precomp, scales, rotations, cov3D_precomp):
        """_RasterizeGaussians.forward_count (old __init__.py:150-199): (gaussians_count, important_score,
        color, radii); no autograd.  `shs` is the full feature tensor (dc first), or dc + the rest separately."""
        rs = self.raster_settings
        if shs is not None and dc is not None and dc.numel():
            shs = torch.cat([dc, shs], dim=1)
        e = _empty_like_device(means3D)
        count, score, _, color, radii, _, _, _ = _C.count_gaussians(
            rs.bg, means3D, e if colors_precomp is None else colors_precomp, opacities,
            e if scales is None else scales, e if rotations is None else rotations, rs.scale_modifier,
            e if cov3D_precomp is None else cov3D_precomp, rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy,
            rs.image_height, rs.image_width, e if shs is None else shs, rs.sh_degree, rs.campos, rs.prefiltered,
            rs.debug, True, getattr(rs, "antialiasing", False))
        return count, score, color, radii

    def visible_filter(self, means3D, scales=None, rotations=None, cov3D_precomp=None):
        rs = self.raster_settings
        e = _empty_like_device(means3D)
        with torch.no_grad():
            return _C.rasterize_gaussians_filter(
                means3D, e if scales is None else scales, e if rotations is None else rotations, rs.scale_modifier,
                e if cov3D_precomp is None else cov3D_precomp, rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy,
                rs.image_height, rs.image_width, rs.prefiltered, rs.debug)


class SparseGaussianAdam(torch.optim.Adam):
    """Adam restricted to visible Gaussians (__init__.py:303-332, adam.cu): b1/b2 fixed at 0.9/0.999, no bias
    correction.  All groups are updated by one launch (dg_adam_update_groups) instead of one adamUpdate per group;
    `stats` (optional, see _C.adam_update_groups) folds the view's densification statistics into the same launch."""

    def __init__(self, params, lr, eps):
        super().__init__(params=params, lr=lr, eps=eps)

    @torch.no_grad()
    def step(self, visibility, N, stats=None, prox=None):
        """prox (optional): {group name: (u, z, coef)} -- an ADMM block trainer's penalty gradient folded into the
        same launch (_C.adam_update_groups)."""
        groups = []
        proxes = []
        for group in self.param_groups:
            lr = group["lr"]
            eps = group["eps"]
            assert len(group["params"]) == 1, "more than one tensor in group"
            param = group["params"][0]
            if param.grad is None:
                continue
            state = self.state[param]
            if len(state) == 0:
                state["step"] = torch.tensor(0.0, dtype=torch.float32)
                state["exp_avg"] = torch.zeros_like(param, memory_format=torch.preserve_format)
                state["exp_avg_sq"] = torch.zeros_like(param, memory_format=torch.preserve_format)
            grad = param.grad if param.grad.is_contiguous() else param.grad.contiguous()
            groups.append((param, grad, state["exp_avg"], state["exp_avg_sq"], lr, eps))
            proxes.append(None if prox is None else prox.get(group.get("name")))
        if groups or stats is not None:
            _C.adam_update_groups(groups, visibility, N, 0.9, 0.999, stats,
                                  prox=proxes if prox is not None else None)
