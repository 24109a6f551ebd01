"""The photometric L1 term of a training view in one launch each way: `rendered_image.clamp(0, 1)` (the end of
render(), gaussian_render.py:149) and `l1_loss(image, gt)` = mean |image - gt| (gaussian_trainer.py's loss), through
dg_clamp_l1_forward / dg_clamp_l1_backward (optim.hip k_clamp_l1_*).  The clamped image is returned too, so the
SSIM term reads it and its gradient joins the L1 gradient and the clamp mask in the same backward pass."""
from __future__ import annotations

import itertools

import torch

from . import _lib

_STAMPS = itertools.count(1)
_RING = 4096
_RINGS: dict = {}


def _stamp_ring(device) -> torch.Tensor:
    """The zero-stamp words of _RowProd on `device` (zeroed once; stamps start at 1)."""
    r = _RINGS.get(device)
    if r is None:
        r = _RINGS[device] = torch.zeros(_RING, dtype=torch.int32, device=device)
    return r


class _ClampL1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, gt):
        _lib.require_device(img, "image")
        _lib.require_f32_on(img.device, image=img, gt=gt)
        # contiguous and 16-B aligned (a contiguous slice can start mid-vector): the kernel reads float4
        x, g = (t.detach().contiguous() for t in (img, gt))
        x, g = (t if t.data_ptr() % 16 == 0 else t.clone() for t in (x, g))
        if x.shape != g.shape:
            raise RuntimeError(f"clamp_l1: image {tuple(x.shape)} vs gt {tuple(g.shape)}")
        n = x.numel()
        L = _lib.load()
        out = torch.empty_like(x)
        nb = int(L.dg_clamp_l1_blocks(n))
        partial = (torch.empty(nb, dtype=torch.float32, device=x.device) if nb else
                   torch.zeros(1, dtype=torch.float32, device=x.device))   # empty image: 0 / 0 = nan, as torch's mean
        with _lib.device_ctx(x.device):
            _lib.check(L.dg_clamp_l1_forward(n, x.data_ptr(), g.data_ptr(), out.data_ptr(), partial.data_ptr(),
                                             _lib.stream_of(x.device)))
            # the mean in one launch, in a fixed order (torch's partial.sum() / n took two)
            l1 = torch.empty((), dtype=torch.float32, device=x.device)
            _lib.check(L.dg_mean_of_parts(partial.data_ptr(), max(nb, 1), n, l1.data_ptr(), _lib.stream_of(x.device)))
        ctx.save_for_backward(x, out, g)
        ctx.set_materialize_grads(False)   # an unused output's gradient stays None (NULL to the kernel), not a fill
        return out, l1

    @staticmethod
    def backward(ctx, g_out, g_l1):
        x, out, g = ctx.saved_tensors
        d = torch.empty_like(x)
        go = None if g_out is None else g_out.contiguous()
        gl = None if g_l1 is None else g_l1.reshape(1).to(torch.float32).contiguous()
        with _lib.device_ctx(x.device):
            _lib.check(_lib.load().dg_clamp_l1_backward(x.numel(), x.data_ptr(), out.data_ptr(), g.data_ptr(),
                                                        None if go is None else go.data_ptr(),
                                                        None if gl is None else gl.data_ptr(), d.data_ptr(),
                                                        _lib.stream_of(x.device)))
        return d, None


def clamp_l1(image: torch.Tensor, gt: torch.Tensor):
    """(image.clamp(0, 1), mean |image.clamp(0, 1) - gt|), both differentiable w.r.t. image."""
    return _ClampL1.apply(image, gt)


class _RowProd(torch.autograd.Function):
    """torch.prod(x, dim=1) for x [N, M <= 3] through dg_row_prod_forward / dg_row_prod_backward: the same values and
    gradients as torch's, without prod_backward's host read of the zero count (a stream sync in the middle of every
    training backward; the kernels keep the zero test on the device: the forward stamps a device word with the call's
    stamp when some element is 0, the backward compares it with the same stamp).  The words are a persistent,
    zero-initialised ring per device (call i uses word i mod 4096 with stamp i): a word only ever holds the stamp of an
    earlier call of its slot, so stale memory cannot match, and up to 4096 forwards may await their
    backward."""

    @staticmethod
    def forward(ctx, x):
        _lib.require_device(x, "x")
        _lib.require_f32_on(x.device, x=x)
        if x.dim() != 2 or not 1 <= x.size(1) <= 3:
            raise RuntimeError(f"row_prod: x must be [N, M] with 1 <= M <= 3, got {tuple(x.shape)}")
        xc = x.detach().contiguous()
        n, m = int(xc.size(0)), int(xc.size(1))
        prod = torch.empty(n, dtype=torch.float32, device=x.device)
        i = next(_STAMPS)
        stamp = i & 0xFFFFFFFF or 1
        flag = _stamp_ring(x.device)[i % _RING:i % _RING + 1]
        with _lib.device_ctx(x.device):
            _lib.check(_lib.load().dg_row_prod_forward(n, m, xc.data_ptr(), prod.data_ptr(), flag.data_ptr(), stamp,
                                                       _lib.stream_of(x.device)))
        ctx.save_for_backward(xc, prod, flag)
        ctx.stamp = stamp
        return prod

    @staticmethod
    def backward(ctx, g):
        xc, prod, flag = ctx.saved_tensors
        n, m = int(xc.size(0)), int(xc.size(1))
        gc = g.contiguous()
        dx = torch.empty_like(xc)
        with _lib.device_ctx(xc.device):
            _lib.check(_lib.load().dg_row_prod_backward(n, m, xc.data_ptr(), prod.data_ptr(), gc.data_ptr(),
                                                        flag.data_ptr(), ctx.stamp, dx.data_ptr(),
                                                        _lib.stream_of(xc.device)))
        return dx


def row_prod(x: torch.Tensor) -> torch.Tensor:
    """x.prod(dim=1) for [N, M <= 3] float32 device tensors (the scale regulariser lambda_scale *
    get_scaling.prod(dim=1).mean(), gaussian_trainer.py:405-408), bit-identical to torch's values and gradients."""
    return _RowProd.apply(x)
