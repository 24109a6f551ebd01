"""Drop-in `fused_ssim` (reference submodules/fused-ssim/fused_ssim/__init__.py:1-41) on MI355X."""
from __future__ import annotations

import torch

from ._cuda import fusedssim, fusedssim_backward, fusedssim_mean, fusedssim_mean_backward

allowed_padding = ["same", "valid"]


class FusedSSIMMap(torch.autograd.Function):
    @staticmethod
    def forward(ctx, C1, C2, img1, img2, padding="same", train=True):
        ssim_map, dm_dmu1, dm_dsigma1_sq, dm_dsigma12 = fusedssim(C1, C2, img1, img2, train)
        if padding == "valid":
            ssim_map = ssim_map[:, :, 5:-5, 5:-5]
        ctx.save_for_backward(img1.detach(), img2, dm_dmu1, dm_dsigma1_sq, dm_dsigma12)
        ctx.C1, ctx.C2, ctx.padding = C1, C2, padding
        return ssim_map

    @staticmethod
    def backward(ctx, opt_grad):
        img1, img2, dm_dmu1, dm_dsigma1_sq, dm_dsigma12 = ctx.saved_tensors
        dL_dmap = opt_grad
        if ctx.padding == "valid":
            dL_dmap = torch.zeros_like(img1)
            dL_dmap[:, :, 5:-5, 5:-5] = opt_grad
        grad = fusedssim_backward(ctx.C1, ctx.C2, img1, img2, dL_dmap, dm_dmu1, dm_dsigma1_sq, dm_dsigma12)
        return None, None, grad, None, None, None


class FusedSSIMMean(torch.autograd.Function):
    """FusedSSIMMap(...).mean() for padding "same" as one Function: the forward totals the map in the kernel (no map, no
    mean reduction launch) and the backward takes the mean's scalar gradient (no materialised dL/dmap, which torch's
    mean backward would expand into a full image first).  Same value as the native training step's SSIM term; the same
    gradient as the map route (dL/dmap = g / numel)."""

    @staticmethod
    def forward(ctx, C1, C2, img1, img2, train=True):
        mean, dm_dmu1, dm_dsigma1_sq, dm_dsigma12 = fusedssim_mean(C1, C2, img1, img2, train)
        ctx.save_for_backward(img1.detach(), img2, dm_dmu1, dm_dsigma1_sq, dm_dsigma12)
        return mean

    @staticmethod
    def backward(ctx, opt_grad):
        img1, img2, dm_dmu1, dm_dsigma1_sq, dm_dsigma12 = ctx.saved_tensors
        grad = fusedssim_mean_backward(img1, img2, opt_grad, dm_dmu1, dm_dsigma1_sq, dm_dsigma12)
        return None, None, grad, None, None


def fused_ssim(img1, img2, padding="same", train=True):
    C1 = 0.01 ** 2
    C2 = 0.03 ** 2
    assert padding in allowed_padding
    if padding == "same":
        return FusedSSIMMean.apply(C1, C2, img1, img2, train)
    return FusedSSIMMap.apply(C1, C2, img1, img2, padding, train).mean()


__all__ = ["fused_ssim", "FusedSSIMMap", "FusedSSIMMean", "fusedssim", "fusedssim_backward", "allowed_padding"]
