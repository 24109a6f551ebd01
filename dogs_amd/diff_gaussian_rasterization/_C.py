"""The `_C` function table of diff_gaussian_rasterization (reference ext.cpp:15-23), implemented over the
C ABI of libdogs_hip.so.  Same names, argument order, return tuples and error behaviour as the
pybind11 functions in rasterize_points.cu; tensors are torch tensors on a HIP device."""
from __future__ import annotations

import contextlib
import ctypes as C
import itertools
import math
import os
import threading

import torch

from .. import _lib

_EMPTY_U8 = None

# Depth-prefix binning policy (dg_raster_args.prefix_per_tile): phase-1 capacity = this x tiles in tile-rect area
# units; 0 -> the library's adaptive capacity (448 per tile, grown while views keep needing phase 2), < 0 -> bin every
# instance in one phase.  Module-level so that the forward and the backward of a view always agree; tests lower it to exercise the phase-2 path.  DOGS_PREFIX_PER_TILE sets it
# for experiments (tools/prefix_sweep.sh).
PREFIX_PER_TILE = int(os.environ.get("DOGS_PREFIX_PER_TILE", "0"))


def set_prefix_per_tile(n: int) -> int:
    global PREFIX_PER_TILE
    old, PREFIX_PER_TILE = PREFIX_PER_TILE, int(n)
    return old


# The adaptive capacity's context (dg_raster_args.capacity_ctx): 0 is the process-wide state; a trainer renders under
# its own (`capacity_context`), so its capacity history -- and with it the instance numbering, hence the rounding of
# its per-Gaussian gradient sums -- depends only on its own views, not on what else the process rendered before (the
# ADMM sequential baseline trains every block in one process; a rank trains one).  Thread-local: the autograd
# engine's backward thread does not read it (the backward carves the capacity the forward returned).
_CTX = threading.local()
_NEXT_CTX = itertools.count(1)


def new_capacity_context(owner=None) -> int:
    """A fresh capacity context; with `owner`, its library state is released when the owner is garbage collected
    (dg_release_capacity_context: the per-context device probes do not outlive the trainer)."""
    ctx = next(_NEXT_CTX)
    if owner is not None:
        import weakref
        weakref.finalize(owner, _lib.release_capacity_context, ctx)
    return ctx


@contextlib.contextmanager
def capacity_context(ctx: int):
    old = getattr(_CTX, "v", 0)
    _CTX.v = int(ctx)
    try:
        yield
    finally:
        _CTX.v = old


def current_capacity_context() -> int:
    return getattr(_CTX, "v", 0)


def _f32(t: torch.Tensor | None) -> torch.Tensor | None:
    if t is None or t.numel() == 0:
        return None
    return t.contiguous() if t.dtype == torch.float32 else t.float().contiguous()


def _args(P, D, M, W, H, bg, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
          viewmatrix, projmatrix, tan_fovx, tan_fovy, dc, sh, campos, prefiltered, antialiasing, debug):
    a = _lib.DgRasterArgs()
    a.P, a.D, a.M, a.W, a.H = int(P), int(D), int(M), int(W), int(H)
    a.prefiltered, a.antialiasing, a.debug = int(bool(prefiltered)), int(bool(antialiasing)), int(bool(debug))
    a.prefix_per_tile = int(PREFIX_PER_TILE)
    a.capacity_ctx = getattr(_CTX, "v", 0)
    a.scale_modifier, a.tanfovx, a.tanfovy = float(scale_modifier), float(tan_fovx), float(tan_fovy)
    keep = dict(bg=_f32(bg), means3D=_f32(means3D), colors=_f32(colors), opacities=_f32(opacity),
                scales=_f32(scales), rotations=_f32(rotations), cov3D_precomp=_f32(cov3D_precomp),
                viewmatrix=_f32(viewmatrix), projmatrix=_f32(projmatrix), dc=_f32(dc), sh=_f32(sh),
                campos=_f32(campos))
    for k, v in keep.items():
        setattr(a, k, _lib.ptr(v))
    return a, keep


def _sh_m(sh: torch.Tensor) -> int:
    return int(sh.size(1)) if sh is not None and sh.dim() >= 2 and sh.size(0) != 0 else 0


def rasterize_gaussians(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                        viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, dc, sh, degree,
                        campos, prefiltered, antialiasing, debug):
    """RasterizeGaussiansCUDA (rasterize_points.cu:55-154)."""
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    _lib.require_device(means3D, "means3D")
    dev = means3D.device
    P, H, W = int(means3D.size(0)), int(image_height), int(image_width)
    fopt = dict(dtype=torch.float32, device=dev)
    u8 = dict(dtype=torch.uint8, device=dev)
    if P == 0:
        return (0, 0, torch.zeros((3, H, W), **fopt), torch.zeros((1, H, W), **fopt),
                torch.zeros((0,), dtype=torch.int32, device=dev), torch.empty(0, **u8), torch.empty(0, **u8),
                torch.empty(0, **u8), torch.empty(0, **u8))
    M = _sh_m(sh)
    with _lib.device_ctx(dev):
        out_color = torch.empty((3, H, W), **fopt)
        out_invdepth = torch.empty((1, H, W), **fopt)
        radii = torch.empty((P,), dtype=torch.int32, device=dev)
        a, keep = _args(P, degree, M, W, H, background, means3D, colors, opacity, scales, rotations, scale_modifier,
                        cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dc, sh, campos, prefiltered,
                        antialiasing, debug)
        arena = _lib.TensorArena(dev)
        gp, bp, ip, b2p = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_void_p()
        nr, nk = C.c_int64(0), C.c_int64(0)
        _lib.check(_lib.load().dg_rasterize_forward(
            C.byref(a), out_color.data_ptr(), out_invdepth.data_ptr(), radii.data_ptr(), arena.fn, None,
            C.byref(gp), C.byref(bp), C.byref(ip), C.byref(b2p), C.byref(nr), C.byref(nk), _lib.stream_of(dev)))
        del keep
    # the reference's sampleBuffer slot carries the phase-2 binning block (empty when phase 2 did not run)
    return (int(nr.value), int(nk.value), out_color, out_invdepth, radii, arena.get(_lib.DG_BUF_GEOM),
            arena.get(_lib.DG_BUF_BINNING), arena.get(_lib.DG_BUF_IMAGE),
            arena.get(_lib.DG_BUF_BINNING2) if b2p.value else torch.empty(0, **u8))


def rasterize_gaussians_backward(background, means3D, radii, colors, opacities, scales, rotations, scale_modifier,
                                 cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color, dc, sh,
                                 dL_dout_invdepth, degree, campos, geomBuffer, R, binningBuffer, imageBuffer, B,
                                 sampleBuffer, antialiasing, debug):
    """RasterizeGaussiansBackwardCUDA (rasterize_points.cu:157-252).  B is the token the forward returned in the
    num_buckets slot (the phase-1 binning capacity of that view)."""
    _lib.require_device(means3D, "means3D")
    dev = means3D.device
    P = int(means3D.size(0))
    H, W = int(dL_dout_color.size(1)), int(dL_dout_color.size(2))
    M = _sh_m(sh)
    fopt = dict(dtype=torch.float32, device=dev)
    if P == 0:
        z = lambda *s: torch.zeros(s, **fopt)  # noqa: E731
        return (z(0, 3), z(0, 3), z(0, 1), z(0, 3), z(0, 6), z(0, 1, 3), z(0, M, 3), z(0, 3), z(0, 4), z(0, 1))
    with _lib.device_ctx(dev):
        # one buffer, outputs back to back in the C ABI's order: the library zero-fills it with a single memset
        shapes = [(P, 3), (P, 3), (P, 1), (P, 3), (P, 6), (P, 1, 3), (P, M, 3), (P, 3), (P, 4), (P, 1)]
        sizes = [math.prod(sh) for sh in shapes]
        buf = torch.empty(sum(sizes), **fopt)
        dmeans2D, dcolors, dopacity, dmeans3D, dcov3D, ddc, dsh, dscales, drot, depth = (
            t.view(sh) for t, sh in zip(torch.split(buf, sizes), shapes))
        a, keep = _args(P, degree, M, W, H, background, means3D, colors, opacities, scales, rotations, scale_modifier,
                        cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dc, sh, campos, False,
                        antialiasing, debug)
        gc = _f32(dL_dout_color)
        gi = _f32(dL_dout_invdepth) if dL_dout_invdepth is not None else None
        radii_c = radii.contiguous()
        arena = _lib.TensorArena(dev)
        _lib.check(_lib.load().dg_rasterize_backward(
            C.byref(a), radii_c.data_ptr(), geomBuffer.data_ptr(), binningBuffer.data_ptr(), imageBuffer.data_ptr(),
            _lib.ptr(sampleBuffer), int(R), int(B), gc.data_ptr(), _lib.ptr(gi), dmeans2D.data_ptr(), dcolors.data_ptr(),
            dopacity.data_ptr(), dmeans3D.data_ptr(), dcov3D.data_ptr(), ddc.data_ptr(), _lib.ptr(dsh),
            dscales.data_ptr(), drot.data_ptr(), depth.data_ptr(), arena.fn, None, _lib.stream_of(dev)))
        del keep
    return dmeans2D, dcolors, dopacity, dmeans3D, dcov3D, ddc, dsh, dscales, drot, depth


_PLAN_LOCK = threading.Lock()
_EAGER_PLANS: dict = {}      # device -> number of plans holding their buffers ahead of the backward


class BackwardPlan:
    """What rasterize_gaussians_backward builds before its C call -- the argument struct, the ten gradient outputs (one
    buffer) and the DG_BUF_BACKWARD scratch (through dg_fixed_alloc, no allocation callback) -- made by the autograd
    forward right after its C call returns, while the GPU renders and the host would otherwise wait: the backward
    (rasterize_gaussians_backward_planned) is then one C call, and the GPU does not idle while Python prepares it.

    Only the argument struct and the sizes are always made in the forward.  The buffers (about 0.9 GB for a 1e6-Gaussian
    1080p view) are allocated there only while no other plan on the device holds its buffers ("eager"): the training
    loop's forward -> backward alternation keeps the hidden host work, while a caller that renders several grad-mode
    views before one backward, or keeps a grad-mode render for metrics, holds at most one view's buffers ahead of
    time -- the other plans allocate in their backward, as the reference does.  An eager plan hands its slot back when
    its backward ran or when it is dropped with its autograd graph."""
    __slots__ = ("a", "keep", "outs", "scratch", "fixed", "P", "M", "nbytes", "dev", "eager", "__weakref__")

    def allocate(self) -> None:
        if self.outs is not None:
            return
        P, M = self.P, self.M
        shapes = [(P, 3), (P, 3), (P, 1), (P, 3), (P, 6), (P, 1, 3), (P, M, 3), (P, 3), (P, 4), (P, 1)]
        sizes = [math.prod(sh) for sh in shapes]
        with _lib.device_ctx(self.dev):
            buf = torch.empty(sum(sizes), dtype=torch.float32, device=self.dev)
            self.outs = tuple(t.view(sh) for t, sh in zip(torch.split(buf, sizes), shapes))
            self.scratch = torch.empty(max(self.nbytes, 1), dtype=torch.uint8, device=self.dev)
        self.fixed = _lib.DgFixedBuffer(self.scratch.data_ptr(), self.nbytes)

    def release(self) -> None:
        """Drop the scratch (the outputs belong to the caller once returned) and the eager slot."""
        self.scratch = self.fixed = None
        if self.eager:
            self.eager = False
            with _PLAN_LOCK:
                _EAGER_PLANS[self.dev] -= 1

    def __del__(self):
        try:
            self.release()
        except Exception:   # interpreter shutdown
            pass


def eager_plans(device) -> int:
    """Plans on `device` whose buffers are allocated ahead of their backward (0 or 1)."""
    with _PLAN_LOCK:
        return _EAGER_PLANS.get(torch.device(device), 0)


def backward_plan(background, means3D, colors, opacities, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
                  projmatrix, tan_fovx, tan_fovy, image_height, image_width, dc, sh, degree, campos, antialiasing, debug,
                  num_rendered):
    """A BackwardPlan for the forward just made with these arguments (num_rendered: its return), or None (P = 0)."""
    P = int(means3D.size(0))
    if P == 0:
        return None
    dev = means3D.device
    pl = BackwardPlan()
    pl.P, pl.M, pl.dev, pl.eager = P, _sh_m(sh), dev, False
    pl.outs = pl.scratch = pl.fixed = None
    with _lib.device_ctx(dev):
        pl.a, pl.keep = _args(P, degree, pl.M, int(image_width), int(image_height), background, means3D, colors,
                              opacities, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix, projmatrix,
                              tan_fovx, tan_fovy, dc, sh, campos, False, antialiasing, debug)
        pl.nbytes = int(_lib.load().dg_backward_scratch_bytes(C.byref(pl.a), int(num_rendered)))
    with _PLAN_LOCK:
        if _EAGER_PLANS.get(dev, 0) == 0:
            _EAGER_PLANS[dev] = 1
            pl.eager = True
    if pl.eager:
        pl.allocate()
    return pl


def rasterize_gaussians_backward_planned(plan, radii, dL_dout_color, dL_dout_invdepth, geomBuffer, R, binningBuffer,
                                         imageBuffer, B, sampleBuffer):
    """rasterize_gaussians_backward with a BackwardPlan: the same C call and outputs (dmeans2D, dcolors, dopacity,
    dmeans3D, dcov3D, ddc, dsh, dscales, drot, depth); dL_dout_invdepth may be None (zeros)."""
    dev = radii.device
    gc = _f32(dL_dout_color)
    gi = _f32(dL_dout_invdepth) if dL_dout_invdepth is not None else None
    plan.allocate()
    o = plan.outs
    _lib.check(_lib.load().dg_rasterize_backward(
        C.byref(plan.a), radii.data_ptr(), geomBuffer.data_ptr(), binningBuffer.data_ptr(), imageBuffer.data_ptr(),
        _lib.ptr(sampleBuffer), int(R), int(B), gc.data_ptr(), _lib.ptr(gi), o[0].data_ptr(), o[1].data_ptr(),
        o[2].data_ptr(), o[3].data_ptr(), o[4].data_ptr(), o[5].data_ptr(), _lib.ptr(o[6]), o[7].data_ptr(),
        o[8].data_ptr(), o[9].data_ptr(), _lib.fixed_alloc_fn(), C.byref(plan.fixed), _lib.stream_of(dev)))
    plan.release()
    return o


def mark_visible(means3D, viewmatrix, projmatrix):
    """markVisible (rasterize_points.cu:254-273)."""
    _lib.require_device(means3D, "means3D")
    P = int(means3D.size(0))
    present = torch.zeros((P,), dtype=torch.bool, device=means3D.device)
    if P:
        m, v, p = _f32(means3D), _f32(viewmatrix), _f32(projmatrix)
        with _lib.device_ctx(means3D.device):
            _lib.check(_lib.load().dg_mark_visible(P, m.data_ptr(), v.data_ptr(), p.data_ptr(), present.data_ptr(),
                                                   _lib.stream_of(means3D.device)))
    return present


def count_gaussians(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                    viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                    prefiltered, debug, f_count=True, antialiasing=False):
    """CountGaussiansCUDA of old_diff-gaussian-rasterization (rasterize_points.cu:148-233; ext.cpp:19), the
    LightGaussian count forward: returns (gaussians_count int32[P], important_score float[P], num_rendered,
    color[3,H,W], radii, geomBuffer, binningBuffer, imgBuffer).  `sh` holds the full SH features [P,(D+1)^2,3]
    (dc first) as in the old binding.  The private buffers are not needed after this call (empty tensors)."""
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    _lib.require_device(means3D, "means3D")
    dev = means3D.device
    P, H, W = int(means3D.size(0)), int(image_height), int(image_width)
    fopt = dict(dtype=torch.float32, device=dev)
    u8 = dict(dtype=torch.uint8, device=dev)
    color = torch.zeros((3, H, W), **fopt)
    radii = torch.zeros((P,), dtype=torch.int32, device=dev)
    count = torch.zeros((P,), dtype=torch.int32, device=dev)
    score = torch.zeros((P,), **fopt)
    nr = C.c_int64(0)
    if P:
        dc = rest = None
        if sh is not None and sh.numel() and sh.dim() == 3 and sh.size(0) == P:
            dc, rest = sh[:, :1, :], sh[:, 1:, :]
        M = _sh_m(rest) if rest is not None else 0
        with _lib.device_ctx(dev):
            a, keep = _args(P, degree, M, W, H, background, means3D, colors, opacity, scales, rotations,
                            scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dc, rest, campos,
                            prefiltered, antialiasing, debug)
            arena = _lib.TensorArena(dev)
            _lib.check(_lib.load().dg_rasterize_count(C.byref(a), color.data_ptr(), radii.data_ptr(), count.data_ptr(),
                                                      score.data_ptr(), arena.fn, None, C.byref(nr),
                                                      _lib.stream_of(dev)))
            del keep
    e = torch.empty(0, **u8)
    return count, score, int(nr.value), color, radii, e, e, e


def rasterize_gaussians_filter(means3D, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix, projmatrix,
                               tan_fovx, tan_fovy, image_height, image_width, prefiltered, debug):
    """RasterizeGaussiansFilterCUDA (rasterize_points.cu:276-334)."""
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    _lib.require_device(means3D, "means3D")
    dev = means3D.device
    P = int(means3D.size(0))
    radii = torch.zeros((P,), dtype=torch.int32, device=dev)
    if P:
        a, keep = _args(P, 0, 0, image_width, image_height, None, means3D, None, None, scales, rotations,
                        scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, None, None, None,
                        prefiltered, False, debug)
        with _lib.device_ctx(dev):
            _lib.check(_lib.load().dg_rasterize_filter(C.byref(a), radii.data_ptr(), _lib.stream_of(dev)))
        del keep
    return radii


def adamUpdate(param, param_grad, exp_avg, exp_avg_sq, visible, lr, b1, b2, eps, N, M):  # noqa: N802
    """adamUpdate (rasterize_points.cu:336-361): in place on param / exp_avg / exp_avg_sq."""
    for t, n in ((param, "param"), (param_grad, "param_grad"), (exp_avg, "exp_avg"), (exp_avg_sq, "exp_avg_sq")):
        _lib.require_device(t, n)
        if not t.is_contiguous() or t.dtype != torch.float32:
            raise RuntimeError(f"{n} must be a contiguous float32 tensor (updated in place)")
    vis = visible.contiguous()
    if vis.dtype != torch.bool:
        vis = vis.bool()
    with _lib.device_ctx(param.device):
        _lib.check(_lib.load().dg_adam_update(param.data_ptr(), param_grad.data_ptr(), exp_avg.data_ptr(),
                                              exp_avg_sq.data_ptr(), vis.data_ptr(), float(lr), float(b1), float(b2),
                                              float(eps), int(N), int(M), _lib.stream_of(param.device)))


def fusedssim(C1, C2, img1, img2):
    """conv.cu fusedssim (exported by the reference _C, unused by conerf): img [3,H,W] -> SSIM map."""
    from ..fused_ssim import _cuda
    m = _cuda.fusedssim(C1, C2, img1.unsqueeze(0), img2.unsqueeze(0), False)[0]
    return m[0]


def fusedssim_backward(C1, C2, img1, img2, dL_dmap):
    """conv.cu fusedssim_backward: recomputes the partial maps, then the fused backward."""
    from ..fused_ssim import _cuda
    a, b = img1.unsqueeze(0), img2.unsqueeze(0)
    _, d1, d2, d3 = _cuda.fusedssim(C1, C2, a, b, True)
    return _cuda.fusedssim_backward(C1, C2, a, b, dL_dmap.unsqueeze(0), d1, d2, d3)[0]


def _check_group(param, grad, m, v):
    for t, n in ((param, "param"), (grad, "grad"), (m, "exp_avg"), (v, "exp_avg_sq")):
        _lib.require_device(t, n)
        if not t.is_contiguous() or t.dtype != torch.float32:
            raise RuntimeError(f"{n} must be a contiguous float32 tensor")


# The group table of the last few group sets (a training loop passes the same parameters, moments and -- from the
# caching allocator -- usually the same gradient addresses every step): building and checking it was ~90 us of host
# per step, more than the launch.  Keyed by every pointer and size it holds (the learning rate and eps are rewritten on
# every call: the xyz rate follows its schedule) and every dtype and device, so a tensor that reuses a freed address
# with another dtype (fp16 moments, bf16 gradients) misses the cache and fails the float32 check; contiguity is
# checked on every call (a view can share a pointer).
_GROUP_TABLES: dict = {}


def _group_array(chunk, N):
    key = (int(N),) + tuple((p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(), g.numel(), m.numel(),
                             v.numel(), p.dtype, g.dtype, m.dtype, v.dtype, p.device, g.device, m.device, v.device)
                            for p, g, m, v, _, _ in chunk)
    arr = _GROUP_TABLES.get(key)
    if arr is not None:
        for i, (p, g, m, v, lr, eps) in enumerate(chunk):
            if not (p.is_contiguous() and g.is_contiguous() and m.is_contiguous() and v.is_contiguous()):
                _check_group(p, g, m, v)  # raises with the tensor's name
            arr[i].lr = float(lr)         # the learning rates follow their schedules step by step
            arr[i].eps = float(eps)
        return arr
    arr = (_lib.DgAdamGroup * max(1, len(chunk)))()
    for i, (param, grad, m, v, lr, eps) in enumerate(chunk):
        _check_group(param, grad, m, v)
        arr[i] = _lib.DgAdamGroup(param.data_ptr(), grad.data_ptr(), m.data_ptr(), v.data_ptr(), float(lr),
                                  float(eps), int(param.numel() // N) if N else 0)
    if len(_GROUP_TABLES) >= 16:
        _GROUP_TABLES.clear()
    _GROUP_TABLES[key] = arr
    return arr


def adam_update_groups(groups, visible, N, b1=0.9, b2=0.999, stats=None, prox=None):
    """SparseGaussianAdam over several groups in one launch (dg_adam_update_groups; each group as adamUpdate).
    groups: iterable of (param, grad, exp_avg, exp_avg_sq, lr, eps); stats (optional): dict with radii [N] int32,
    dmeans2D [N,>=2] (screen-space-point gradient), max_radii2D [N], grad_accum [N(,1)], denom [N(,1)] -- the view's
    densification statistics (gaussian_trainer.py:433-438), updated in the same launch.  prox (optional): one entry
    per group, None or (u, z, coef) -- the ADMM penalty 0.5 rho mse(x + u, z) of a block trainer as its gradient
    coef ((x + u) - z), coef = rho / numel(x), added for the rows Adam updates (dg_adam_update_groups_prox)."""
    groups = list(groups)
    prox = list(prox) if prox is not None else None
    if prox is not None and len(prox) != len(groups):
        raise RuntimeError("prox needs one entry (or None) per group")
    vis = visible.contiguous()
    if vis.dtype != torch.bool:
        vis = vis.bool()
    dev = vis.device
    keep = [vis]
    arr = (_lib.DgAdamGroup * max(1, min(8, len(groups))))()
    st = None
    if stats is not None:
        dm = stats["dmeans2D"]
        if dm.dim() != 2 or dm.stride(1) != 1 or dm.size(1) < 2:
            dm = dm.reshape(int(N), -1).contiguous()
        for k in ("max_radii2D", "grad_accum", "denom"):
            t = stats[k]
            if not t.is_contiguous() or t.dtype != torch.float32:
                raise RuntimeError(f"{k} must be a contiguous float32 tensor (updated in place)")
        radii = stats["radii"].contiguous()
        if radii.dtype != torch.int32:
            radii = radii.int()
        keep += [dm, radii]
        st = _lib.DgDensifyStats(radii.data_ptr(), dm.data_ptr(), int(dm.stride(0)), stats["max_radii2D"].data_ptr(),
                                 stats["grad_accum"].data_ptr(), stats["denom"].data_ptr())
    L = _lib.load()
    parr = (_lib.DgAdamProx * max(1, min(8, len(groups))))() if prox is not None else None
    with _lib.device_ctx(dev):
        for c0 in range(0, max(1, len(groups)), 8):
            chunk = groups[c0:c0 + 8]
            if parr is None:
                arr = _group_array(chunk, N)
            else:
                for i, (param, grad, m, v, lr, eps) in enumerate(chunk):
                    _check_group(param, grad, m, v)
                    arr[i] = _lib.DgAdamGroup(param.data_ptr(), grad.data_ptr(), m.data_ptr(), v.data_ptr(),
                                              float(lr), float(eps), int(param.numel() // N) if N else 0)
                    pe = prox[c0 + i]
                    if pe is None:
                        parr[i] = _lib.DgAdamProx(None, None, 0.0)
                    else:
                        u, z, coef = pe
                        for t, n in ((u, "dual"), (z, "global")):
                            _lib.require_f32_on(param.device, **{n: t})
                            if not t.is_contiguous() or t.shape != param.shape:
                                raise RuntimeError(f"{n} must be a contiguous tensor shaped like the parameter")
                        keep += [u, z]
                        parr[i] = _lib.DgAdamProx(u.data_ptr(), z.data_ptr(), float(coef))
            st_p = C.byref(st) if (st is not None and c0 == 0) else None
            if parr is not None:
                _lib.check(L.dg_adam_update_groups_prox(arr, parr, len(chunk), vis.data_ptr(), int(N), float(b1),
                                                        float(b2), st_p, _lib.stream_of(dev)))
            else:
                _lib.check(L.dg_adam_update_groups(arr, len(chunk), vis.data_ptr(), int(N), float(b1), float(b2),
                                                   st_p, _lib.stream_of(dev)))
    del keep
