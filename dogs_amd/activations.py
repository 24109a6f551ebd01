"""The Gaussian parameter activations of a training view in one launch each way: GaussianSplatModel.get_opacity
(sigmoid), get_scaling (exp) and get_quaternion (F.normalize, eps 1e-12) -- conerf/model/gaussian_fields/
gaussian_splat_model.py -- through dg_activate_forward / dg_activate_backward (optim.hip k_activate_*), where torch
launches about four kernels forward and eight backward for the three."""
from __future__ import annotations

import torch

from . import _lib


def _c(t: torch.Tensor) -> torch.Tensor:
    """Contiguous and 16-B aligned (rotation rows are read as float4; a contiguous slice may start mid-row)."""
    t = t.detach().contiguous()
    return t if t.data_ptr() % 16 == 0 else t.clone()


class _Activate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, raw_opacity, raw_scaling, raw_rotation):
        _lib.require_device(raw_opacity, "raw_opacity")
        _lib.require_f32_on(raw_opacity.device, raw_opacity=raw_opacity, raw_scaling=raw_scaling,
                            raw_rotation=raw_rotation)
        ro, rs, rq = _c(raw_opacity), _c(raw_scaling), _c(raw_rotation)
        n = int(ro.shape[0])
        if rs.shape != (n, 3) or rq.shape != (n, 4) or ro.numel() != n:
            raise RuntimeError(f"activate: shapes {tuple(ro.shape)}, {tuple(rs.shape)}, {tuple(rq.shape)}")
        o, sc, q = torch.empty_like(ro), torch.empty_like(rs), torch.empty_like(rq)
        with _lib.device_ctx(ro.device):
            _lib.check(_lib.load().dg_activate_forward(n, ro.data_ptr(), rs.data_ptr(), rq.data_ptr(), o.data_ptr(),
                                                       sc.data_ptr(), q.data_ptr(), _lib.stream_of(ro.device)))
        ctx.save_for_backward(o, sc, rq)
        return o, sc, q

    @staticmethod
    def backward(ctx, g_o, g_sc, g_q):
        o, sc, rq = ctx.saved_tensors
        n = int(o.shape[0])
        d_o, d_sc, d_q = torch.empty_like(o), torch.empty_like(sc), torch.empty_like(rq)
        p = lambda t: None if t is None else _c(t).data_ptr()  # noqa: E731
        with _lib.device_ctx(o.device):
            _lib.check(_lib.load().dg_activate_backward(n, o.data_ptr(), sc.data_ptr(), rq.data_ptr(), p(g_o), p(g_sc),
                                                        p(g_q), d_o.data_ptr(), d_sc.data_ptr(), d_q.data_ptr(),
                                                        _lib.stream_of(o.device)))
        return d_o, d_sc, d_q


def activate(raw_opacity: torch.Tensor, raw_scaling: torch.Tensor, raw_rotation: torch.Tensor):
    """(sigmoid(raw_opacity) [N,1], exp(raw_scaling) [N,3], normalize(raw_rotation) [N,4]), differentiable."""
    return _Activate.apply(raw_opacity, raw_scaling, raw_rotation)
