"""`fused_ssim_cuda` extension table (reference fused-ssim/ext.cpp, ssim.cu:368-444) over libdogs_hip.so."""
from __future__ import annotations

import torch

from .. import _lib


def _c(t):
    return t.contiguous() if t.dtype == torch.float32 else t.float().contiguous()


def fusedssim(C1, C2, img1, img2, train=True):
    """-> (ssim_map, dm_dmu1, dm_dsigma1_sq, dm_dsigma12); the three partial maps are empty when not train."""
    _lib.require_device(img1, "img1")
    a, b = _c(img1), _c(img2)
    B, CH, H, W = (int(x) for x in a.shape)
    dev = a.device
    ssim_map = torch.empty_like(a)
    if train:
        d1, d2, d3 = torch.empty_like(a), torch.empty_like(a), torch.empty_like(a)
    else:
        d1 = d2 = d3 = torch.empty(0, device=dev)
    with _lib.device_ctx(dev):
        _lib.check(_lib.load().dg_fused_ssim_forward(B, CH, H, W, float(C1), float(C2), a.data_ptr(), b.data_ptr(),
                                                     ssim_map.data_ptr(), _lib.ptr(d1), _lib.ptr(d2), _lib.ptr(d3),
                                                     _lib.stream_of(dev)))
    return ssim_map, d1, d2, d3


def fusedssim_backward(C1, C2, img1, img2, dL_dmap, dm_dmu1, dm_dsigma1_sq, dm_dsigma12):
    _lib.require_device(img1, "img1")
    if dm_dmu1.numel() == 0:
        raise RuntimeError("fusedssim_backward needs the partial maps of a train=True forward")
    a, b, g = _c(img1), _c(img2), _c(dL_dmap)
    B, CH, H, W = (int(x) for x in a.shape)
    dev = a.device
    out = torch.empty_like(a)
    with _lib.device_ctx(dev):
        _lib.check(_lib.load().dg_fused_ssim_backward(B, CH, H, W, float(C1), float(C2), a.data_ptr(), b.data_ptr(),
                                                      g.data_ptr(), _c(dm_dmu1).data_ptr(),
                                                      _c(dm_dsigma1_sq).data_ptr(), _c(dm_dsigma12).data_ptr(),
                                                      out.data_ptr(), _lib.stream_of(dev)))
    return out


def fusedssim_mean(C1, C2, img1, img2, train=True):
    """The SSIM map's mean without the map (dg_fused_ssim_mean) -> (mean [] tensor, dm_dmu1, dm_dsigma1_sq,
    dm_dsigma12); the partial maps are empty when not train."""
    _lib.require_device(img1, "img1")
    a, b = _c(img1), _c(img2)
    B, CH, H, W = (int(x) for x in a.shape)
    dev = a.device
    L = _lib.load()
    if train:
        d1, d2, d3 = torch.empty_like(a), torch.empty_like(a), torch.empty_like(a)
    else:
        d1 = d2 = d3 = torch.empty(0, device=dev)
    part = torch.empty(int(L.dg_fused_ssim_parts(B, CH, H, W)), dtype=torch.float32, device=dev)
    mean = torch.empty((), dtype=torch.float32, device=dev)
    with _lib.device_ctx(dev):
        _lib.check(L.dg_fused_ssim_mean(B, CH, H, W, float(C1), float(C2), a.data_ptr(), b.data_ptr(), _lib.ptr(d1),
                                        _lib.ptr(d2), _lib.ptr(d3), part.data_ptr(), mean.data_ptr(),
                                        _lib.stream_of(dev)))
    return mean, d1, d2, d3


def fusedssim_mean_backward(img1, img2, dL_dmean, dm_dmu1, dm_dsigma1_sq, dm_dsigma12):
    """dL/dimg1 from the mean's gradient (a device scalar): dL/dmap = dL_dmean / numel is never materialised."""
    _lib.require_device(img1, "img1")
    if dm_dmu1.numel() == 0:
        raise RuntimeError("fusedssim_backward needs the partial maps of a train=True forward")
    a, b = _c(img1), _c(img2)
    g = dL_dmean.reshape(1)
    g = g if g.dtype == torch.float32 else g.float()
    B, CH, H, W = (int(x) for x in a.shape)
    dev = a.device
    out = torch.empty_like(a)
    with _lib.device_ctx(dev):
        _lib.check(_lib.load().dg_fused_ssim_mean_backward(B, CH, H, W, a.data_ptr(), b.data_ptr(), g.data_ptr(),
                                                           dm_dmu1.data_ptr(), dm_dsigma1_sq.data_ptr(),
                                                           dm_dsigma12.data_ptr(), out.data_ptr(),
                                                           _lib.stream_of(dev)))
    return out
