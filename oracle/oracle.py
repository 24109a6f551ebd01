"""ctypes front-end of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
The product path (dogs_amd/) must never import this module.

The C sources restate, line by line, the reference kernels in
/root/reference/submodules/diff-gaussian-rasterization/cuda_rasterizer/{forward,backward,
rasterizer_impl,adam}.cu, fused-ssim/ssim.cu and simple-knn/simple_knn.cu (see the file
headers for the arithmetic conventions).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libgs_oracle.so")
_lib = None

f32p = C.POINTER(C.c_float)
u32p = C.POINTER(C.c_uint32)
i32p = C.POINTER(C.c_int)
u8p = C.POINTER(C.c_uint8)


class GsoParams(C.Structure):
    _fields_ = [
        ("P", C.c_int), ("D", C.c_int), ("M", C.c_int), ("W", C.c_int), ("H", C.c_int),
        ("prefiltered", C.c_int), ("antialiasing", C.c_int),
        ("scale_modifier", C.c_float), ("tanfovx", C.c_float), ("tanfovy", C.c_float),
        ("bg", f32p), ("means3D", f32p), ("colors", f32p), ("opacities", f32p), ("scales", f32p),
        ("rotations", f32p), ("cov3D_precomp", f32p), ("viewmatrix", f32p), ("projmatrix", f32p),
        ("dc", f32p), ("sh", f32p), ("campos", f32p),
    ]


def build() -> str:
    """Compile the oracle with its own Makefile (gcc, no GPU)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        L.gso_forward.restype = C.c_void_p
        L.gso_forward.argtypes = [C.POINTER(GsoParams), f32p, f32p, i32p, i32p]
        L.gso_backward.restype = C.c_int
        L.gso_backward.argtypes = [C.c_void_p] + [f32p] * 14
        L.gso_free.argtypes = [C.c_void_p]
        for n in ("gso_num_rendered", "gso_num_valid", "gso_num_buckets"):
            getattr(L, n).restype = C.c_int64
            getattr(L, n).argtypes = [C.c_void_p]
        L.gso_num_tiles.restype = C.c_int
        L.gso_num_tiles.argtypes = [C.c_void_p]
        L.gso_copy_list.argtypes = [C.c_void_p, u32p, u32p, u32p]
        L.gso_copy_ranges.argtypes = [C.c_void_p, u32p]
        L.gso_copy_geom.argtypes = [C.c_void_p, f32p, f32p, f32p, f32p, f32p, u8p, u32p]
        L.gso_copy_image_state.argtypes = [C.c_void_p, f32p, u32p, u32p]
        L.gso_copy_counts.argtypes = [C.c_void_p, i32p, f32p]
        L.gso_mark_visible.argtypes = [C.c_int, f32p, f32p, f32p, u8p]
        L.gso_filter_radii.argtypes = [C.POINTER(GsoParams), i32p]
        L.gso_adam.argtypes = [f32p, f32p, f32p, f32p, u8p, C.c_float, C.c_float, C.c_float, C.c_float,
                               C.c_uint32, C.c_uint32]
        L.gso_set_threads.argtypes = [C.c_int]
        L.gso_get_threads.restype = C.c_int
        L.gs_crlogf.restype = C.c_float
        L.gs_crlogf.argtypes = [C.c_float]
        L.gso_crlogf_check.restype = C.c_int64
        L.gso_crlogf_check.argtypes = [C.c_uint32, C.c_uint32, f32p, C.c_int64]
        L.gso_cull_log_threshold.argtypes = [C.c_int64, f32p, f32p]
        L.gso_logf_census.restype = C.c_int
        L.gso_logf_census.argtypes = [C.POINTER(GsoParams), C.POINTER(C.c_int64)]
        L.aux_ssim_fwd.argtypes = [C.c_int] * 4 + [C.c_float, C.c_float] + [f32p] * 6
        L.aux_ssim_bwd.argtypes = [C.c_int] * 4 + [f32p] * 7
        L.aux_knn.restype = C.c_int
        L.aux_knn.argtypes = [C.c_int, f32p, f32p, u32p]
        _lib = L
    return _lib


def _f(a):
    if a is None:
        return None
    return np.ascontiguousarray(a, dtype=np.float32)


def _p(a, t=f32p):
    return None if a is None else a.ctypes.data_as(t)


class OracleForward:
    """Holds the oracle's forward state (GeometryState/BinningState/ImageState/SampleState)."""

    def __init__(self, ctx, keep, P, M, W, H, num_tiles):
        self._ctx = ctx
        self._keep = keep
        self.P, self.M, self.W, self.H, self.num_tiles = P, M, W, H, num_tiles

    def __del__(self):
        if getattr(self, "_ctx", None):
            try:
                lib().gso_free(self._ctx)
            except TypeError:  # interpreter shutdown: module globals already cleared
                pass
            self._ctx = None

    @property
    def num_rendered(self):
        return int(lib().gso_num_rendered(self._ctx))

    @property
    def num_valid(self):
        return int(lib().gso_num_valid(self._ctx))

    @property
    def num_buckets(self):
        return int(lib().gso_num_buckets(self._ctx))

    def sorted_list(self):
        n = self.num_valid
        t = np.zeros(max(n, 1), np.uint32)
        i = np.zeros(max(n, 1), np.uint32)
        d = np.zeros(max(n, 1), np.uint32)
        lib().gso_copy_list(self._ctx, _p(t, u32p), _p(i, u32p), _p(d, u32p))
        return t[:n], i[:n], d[:n]

    def ranges(self):
        r = np.zeros((self.num_tiles, 2), np.uint32)
        lib().gso_copy_ranges(self._ctx, _p(r, u32p))
        return r

    def geom(self):
        P = self.P
        out = dict(depths=np.zeros(P, np.float32), means2D=np.zeros((P, 2), np.float32),
                   conic_opacity=np.zeros((P, 4), np.float32), rgb=np.zeros((P, 3), np.float32),
                   cov3D=np.zeros((P, 6), np.float32), clamped=np.zeros((P, 3), np.uint8),
                   tiles_touched=np.zeros(P, np.uint32))
        lib().gso_copy_geom(self._ctx, _p(out["depths"]), _p(out["means2D"]), _p(out["conic_opacity"]),
                            _p(out["rgb"]), _p(out["cov3D"]), _p(out["clamped"], u8p),
                            _p(out["tiles_touched"], u32p))
        return out

    def image_state(self):
        HW = self.W * self.H
        fT = np.zeros(HW, np.float32)
        nc = np.zeros(HW, np.uint32)
        mc = np.zeros(self.num_tiles, np.uint32)
        lib().gso_copy_image_state(self._ctx, _p(fT), _p(nc, u32p), _p(mc, u32p))
        return fT.reshape(self.H, self.W), nc.reshape(self.H, self.W), mc

    def counts(self):
        """LightGaussian count mode: (gaussians_count int32[P], important_score float32[P])."""
        cnt = np.zeros(self.P, np.int32)
        score = np.zeros(self.P, np.float32)
        lib().gso_copy_counts(self._ctx, _p(cnt, i32p), _p(score))
        return cnt, score

    def backward(self, dL_dpix, dL_dinvdepth=None):
        P, M = self.P, self.M
        dL_dpix = _f(dL_dpix)
        dL_dinv = _f(dL_dinvdepth) if dL_dinvdepth is not None else np.zeros((self.H, self.W), np.float32)
        g = dict(dmeans2D=np.zeros((P, 3), np.float32), dconic=np.zeros((P, 4), np.float32),
                 dopacity=np.zeros((P, 1), np.float32), dcolors=np.zeros((P, 3), np.float32),
                 dinvdepth=np.zeros((P, 1), np.float32), dmeans3D=np.zeros((P, 3), np.float32),
                 dcov3D=np.zeros((P, 6), np.float32), ddc=np.zeros((P, 1, 3), np.float32),
                 dsh=np.zeros((P, max(M, 0), 3), np.float32), dscales=np.zeros((P, 3), np.float32),
                 drot=np.zeros((P, 4), np.float32), depth=np.zeros((P, 1), np.float32))
        order = ["dmeans2D", "dconic", "dopacity", "dcolors", "dinvdepth", "dmeans3D", "dcov3D", "ddc",
                 "dsh", "dscales", "drot", "depth"]
        rc = lib().gso_backward(self._ctx, _p(dL_dpix), _p(dL_dinv), *[_p(g[k]) for k in order])
        if rc != 0:
            raise RuntimeError("oracle backward failed")
        return g


def forward(means3D, opacities, viewmatrix, projmatrix, campos, tanfovx, tanfovy, H, W, bg,
            dc=None, sh=None, colors=None, scales=None, rotations=None, cov3D_precomp=None,
            sh_degree=3, scale_modifier=1.0, antialiasing=False, prefiltered=False):
    """Restates _C.rasterize_gaussians.  Arrays are numpy (any float dtype).  Returns
    (color[3,H,W], radii[P], invdepth[1,H,W], state)."""
    means3D = _f(means3D).reshape(-1, 3)
    P = means3D.shape[0]
    keep = dict(means3D=means3D, opacities=_f(opacities).reshape(-1), view=_f(viewmatrix).reshape(16),
                proj=_f(projmatrix).reshape(16), campos=_f(campos).reshape(3), bg=_f(bg).reshape(3),
                dc=_f(dc), sh=_f(sh), colors=_f(colors), scales=_f(scales), rotations=_f(rotations),
                cov3D=_f(cov3D_precomp))
    M = 0 if keep["sh"] is None or keep["sh"].size == 0 else keep["sh"].reshape(P, -1, 3).shape[1]
    for k in ("sh", "colors", "scales", "rotations", "cov3D", "dc"):
        if keep[k] is not None and keep[k].size == 0:
            keep[k] = None
    prm = GsoParams(P=P, D=int(sh_degree), M=M, W=int(W), H=int(H), prefiltered=int(prefiltered),
                    antialiasing=int(antialiasing), scale_modifier=float(scale_modifier),
                    tanfovx=float(tanfovx), tanfovy=float(tanfovy),
                    bg=_p(keep["bg"]), means3D=_p(means3D), colors=_p(keep["colors"]),
                    opacities=_p(keep["opacities"]), scales=_p(keep["scales"]),
                    rotations=_p(keep["rotations"]), cov3D_precomp=_p(keep["cov3D"]),
                    viewmatrix=_p(keep["view"]), projmatrix=_p(keep["proj"]), dc=_p(keep["dc"]),
                    sh=_p(keep["sh"]), campos=_p(keep["campos"]))
    keep["prm"] = prm
    color = np.zeros((3, H, W), np.float32)
    invd = np.zeros((1, H, W), np.float32)
    radii = np.zeros(P, np.int32)
    err = C.c_int(0)
    ctx = lib().gso_forward(C.byref(prm), _p(color), _p(invd), _p(radii, i32p), C.byref(err))
    if not ctx:
        raise RuntimeError(f"oracle forward failed (err={err.value})")
    num_tiles = ((W + 15) // 16) * ((H + 15) // 16)
    st = OracleForward(ctx, keep, P, M, W, H, num_tiles)
    return color, radii, invd, st


def set_threads(n: int) -> int:
    """Threads of the oracle's OpenMP loops (<= 0: all cores); returns the previous count.  Results are
    bit-identical for any count (gs_oracle.c header)."""
    old = int(lib().gso_get_threads())
    lib().gso_set_threads(int(n))
    return old


def get_threads() -> int:
    return int(lib().gso_get_threads())


def mark_visible(means3D, viewmatrix, projmatrix):
    m = _f(means3D).reshape(-1, 3)
    out = np.zeros(m.shape[0], np.uint8)
    lib().gso_mark_visible(m.shape[0], _p(m), _p(_f(viewmatrix).reshape(16)), _p(_f(projmatrix).reshape(16)),
                           _p(out, u8p))
    return out.astype(bool)


def filter_radii(means3D, viewmatrix, projmatrix, tanfovx, tanfovy, H, W, scales=None, rotations=None,
                 cov3D_precomp=None, scale_modifier=1.0):
    m = _f(means3D).reshape(-1, 3)
    keep = [m, _f(scales), _f(rotations), _f(cov3D_precomp), _f(viewmatrix).reshape(16),
            _f(projmatrix).reshape(16)]
    prm = GsoParams(P=m.shape[0], W=int(W), H=int(H), scale_modifier=float(scale_modifier),
                    tanfovx=float(tanfovx), tanfovy=float(tanfovy), means3D=_p(m),
                    scales=_p(keep[1]) if keep[1] is not None and keep[1].size else None,
                    rotations=_p(keep[2]) if keep[2] is not None and keep[2].size else None,
                    cov3D_precomp=_p(keep[3]) if keep[3] is not None and keep[3].size else None,
                    viewmatrix=_p(keep[4]), projmatrix=_p(keep[5]))
    radii = np.zeros(m.shape[0], np.int32)
    lib().gso_filter_radii(C.byref(prm), _p(radii, i32p))
    return radii


def adam(param, grad, m, v, visible, lr, b1, b2, eps, N, M):
    """In-place on numpy float32 arrays (adam.cu:10-38)."""
    vis = np.ascontiguousarray(visible, dtype=np.uint8)
    lib().gso_adam(_p(param), _p(grad), _p(m), _p(v), _p(vis, u8p), lr, b1, b2, eps, N, M)


def ssim_forward(img1, img2, C1=0.01 ** 2, C2=0.03 ** 2, train=True):
    a, b = _f(img1), _f(img2)
    B, CH, H, W = a.shape
    mp = np.zeros_like(a)
    d = [np.zeros_like(a) for _ in range(3)] if train else [None] * 3
    lib().aux_ssim_fwd(B, CH, H, W, C1, C2, _p(a), _p(b), _p(mp), *[_p(x) for x in d])
    return (mp, *d)


def ssim_backward(img1, img2, dL_dmap, dm_dmu1, dm_dsigma1_sq, dm_dsigma12):
    a, b = _f(img1), _f(img2)
    B, CH, H, W = a.shape
    out = np.zeros_like(a)
    lib().aux_ssim_bwd(B, CH, H, W, _p(a), _p(b), _p(_f(dL_dmap)), _p(_f(dm_dmu1)), _p(_f(dm_dsigma1_sq)),
                       _p(_f(dm_dsigma12)), _p(out))
    return out


# fused-ssim's window (ssim.cu:11-15): the float32 constants, held exactly in float64
_SSIM_GW = np.array([0.001028380123898387, 0.0075987582094967365, 0.036000773310661316, 0.10936068743467331,
                     0.21300552785396576, 0.26601171493530273, 0.21300552785396576, 0.10936068743467331,
                     0.036000773310661316, 0.0075987582094967365, 0.001028380123898387], np.float32).astype(np.float64)


def _conv11_f64(x: np.ndarray) -> np.ndarray:
    """The zero-padded separable 11 x 11 Gaussian window over the last two axes, in float64."""
    H, W = x.shape[-2:]
    p = np.pad(x, [(0, 0)] * (x.ndim - 2) + [(5, 5), (5, 5)])
    h = sum(g * p[..., :, k:k + W] for k, g in enumerate(_SSIM_GW))
    return sum(g * h[..., k:k + H, :] for k, g in enumerate(_SSIM_GW))


def ssim_forward_exact(img1, img2, C1=0.01 ** 2, C2=0.03 ** 2):
    """ssim_forward's four maps evaluated in float64 on the same float32 inputs: the value every float32 summation
    order approximates.  A GPU kernel that sums the window in another order than the reference's (ssim.cu:187-286)
    is held to the reference order's own float32 error against this (tests/test_gpu_aux.py)."""
    a, b = _f(img1).astype(np.float64), _f(img2).astype(np.float64)
    mu1, mu2 = _conv11_f64(a), _conv11_f64(b)
    s1 = _conv11_f64(a * a) - mu1 * mu1
    s2 = _conv11_f64(b * b) - mu2 * mu2
    s12 = _conv11_f64(a * b) - mu1 * mu2
    Cc, D = 2 * mu1 * mu2 + C1, 2 * s12 + C2
    A, B = mu1 * mu1 + mu2 * mu2 + C1, s1 + s2 + C2
    d1 = (mu2 * 2 * D) / (A * B) - (mu2 * 2 * Cc) / (A * B) - (mu1 * 2 * Cc * D) / (A * A * B) + \
        (mu1 * 2 * Cc * D) / (A * B * B)
    return Cc * D / (A * B), d1, (-Cc * D) / (A * B * B), (2 * Cc) / (A * B)


def ssim_backward_exact(img1, img2, dL_dmap, dm_dmu1, dm_dsigma1_sq, dm_dsigma12):
    """ssim_backward in float64 on the same float32 inputs (ssim.cu:288-366)."""
    a, b = _f(img1).astype(np.float64), _f(img2).astype(np.float64)
    dl = _f(dL_dmap).astype(np.float64)
    t = [_conv11_f64(_f(x).astype(np.float64) * dl) for x in (dm_dmu1, dm_dsigma1_sq, dm_dsigma12)]
    return t[0] + 2 * a * t[1] + b * t[2]


def knn_dist2(points):
    p = _f(points).reshape(-1, 3)
    out = np.zeros(p.shape[0], np.float32)
    order = np.zeros(p.shape[0], np.uint32)
    if lib().aux_knn(p.shape[0], _p(p), _p(out), _p(order, u32p)) != 0:
        raise RuntimeError("oracle knn failed")
    return out


def gs_crlogf(x: float) -> float:
    """The cull's logf (gs_oracle.c gs_crlogf): correctly rounded on the cull's domain."""
    return float(lib().gs_crlogf(float(x)))


def cull_log_threshold(opacity) -> np.ndarray:
    """logf(opacity / (1/255)) as the precise cull evaluates it (gs_crlogf), per element."""
    o = _f(opacity).reshape(-1)
    out = np.empty_like(o)
    lib().gso_cull_log_threshold(o.size, _p(o), _p(out))
    return out


def crlogf_check(lo_bits: int, hi_bits: int, max_bad: int = 64):
    """gs_crlogf against logl rounded to float over the float bit patterns [lo_bits, hi_bits): (count, inputs)."""
    bad = np.zeros(max(max_bad, 1), np.float32)
    n = int(lib().gso_crlogf_check(lo_bits, hi_bits, _p(bad), max_bad))
    return n, bad[:min(n, max_bad)].copy()


def logf_census(means3D, opacities, viewmatrix, projmatrix, campos, tanfovx, tanfovy, H, W, scales, rotations,
                antialiasing=False):
    """gso_logf_census: the precise cull's keep decisions under round 5's gs_logf and under gs_crlogf."""
    means3D = _f(means3D).reshape(-1, 3)
    keep = dict(o=_f(opacities).reshape(-1), v=_f(viewmatrix).reshape(16), p=_f(projmatrix).reshape(16),
                c=_f(campos).reshape(3), s=_f(scales), r=_f(rotations), bg=np.zeros(3, np.float32),
                col=np.zeros((means3D.shape[0], 3), np.float32))
    prm = GsoParams(P=means3D.shape[0], D=0, M=0, W=int(W), H=int(H), prefiltered=0, antialiasing=int(antialiasing),
                    scale_modifier=1.0, tanfovx=float(tanfovx), tanfovy=float(tanfovy), bg=_p(keep["bg"]),
                    means3D=_p(means3D), colors=_p(keep["col"]),
                    opacities=_p(keep["o"]), scales=_p(keep["s"]), rotations=_p(keep["r"]), cov3D_precomp=None,
                    viewmatrix=_p(keep["v"]), projmatrix=_p(keep["p"]), dc=None, sh=None, campos=_p(keep["c"]))
    out = (C.c_int64 * 6)()
    if lib().gso_logf_census(C.byref(prm), out) != 0:
        raise MemoryError("oracle census: allocation failed")
    keys = ("tested", "kept", "kept_only_r5", "kept_only_cr", "rendered", "threshold_differs")
    return dict(zip(keys, (int(v) for v in out)))
