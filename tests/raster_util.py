"""Shared helpers for rasterizer parity tests: scene construction and oracle/HIP invocation."""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from dogs_amd.synthetic import make_scene


def small_scene(n, W, H, seed=1234, fx=None, sh_rest=15):
    """Synthetic scene (dogs_amd.synthetic) at a small image size; Gaussian scales are enlarged so the
    screen footprint matches the 1080p/fx=1600 north-star scene (median radius ~14 px there)."""
    fx = fx if fx is not None else 0.8 * max(W, H)
    s = make_scene(n, W, H, fx=fx, fy=fx, seed=seed, sh_rest=sh_rest)
    k = float(1600.0 / fx) * (max(W, H) / 1920.0)
    s.scales = (s.scales * k).contiguous()
    s.raw_scales = s.raw_scales + float(np.log(k))
    return s


def oracle_forward(O, s, bg, deg=3, antialiasing=False, colors=None, cov3D=None, scale_modifier=1.0):
    c = s.camera
    kw = dict(dc=None if colors is not None else s.dc.numpy(), sh=None if colors is not None else s.sh.numpy(),
              colors=colors, scales=None if cov3D is not None else s.scales.numpy(),
              rotations=None if cov3D is not None else s.rotations.numpy(), cov3D_precomp=cov3D)
    return O.forward(s.means3D.numpy(), s.opacities.numpy(), c.world_to_camera.numpy(), c.projective_matrix.numpy(),
                     c.camera_center.numpy(), c.tanfovx, c.tanfovy, c.height, c.width, np.asarray(bg, np.float32),
                     sh_degree=deg, antialiasing=antialiasing, scale_modifier=scale_modifier, **kw)


def hip_forward(s, bg, dev, deg=3, antialiasing=False, colors=None, cov3D=None, scale_modifier=1.0, debug=False):
    from dogs_amd.diff_gaussian_rasterization import _C
    c = s.camera.to(dev)
    e = torch.empty(0, device=dev)
    d = lambda t: t.to(dev).contiguous()  # noqa: E731
    out = _C.rasterize_gaussians(
        torch.as_tensor(bg, dtype=torch.float32, device=dev), d(s.means3D),
        e if colors is None else d(torch.as_tensor(colors)), d(s.opacities),
        e if cov3D is not None else d(s.scales), e if cov3D is not None else d(s.rotations), scale_modifier,
        e if cov3D is None else d(torch.as_tensor(cov3D)), c.world_to_camera, c.projective_matrix, c.tanfovx,
        c.tanfovy, c.height, c.width, e if colors is not None else d(s.dc), e if colors is not None else d(s.sh),
        deg, c.camera_center, False, antialiasing, debug)
    return out


def hip_sorted_instances(out, W, H, dev, P):
    """(tiles, gaussians, E1): the phase-1 instances (E1, grouped by tile) followed by the phase-2 ones."""
    import ctypes as C
    from dogs_amd import _lib
    from dogs_amd.diff_gaussian_rasterization import _C
    L = _lib.load()
    nb = C.c_int64(0)
    _lib.check(L.dg_binned_instances(out[5].data_ptr(), int(P), C.byref(nb), _lib.stream_of(dev)))
    K = int(nb.value)
    a = _lib.DgRasterArgs()
    a.P, a.W, a.H, a.prefix_per_tile = int(P), int(W), int(H), int(_C.PREFIX_PER_TILE)
    tiles = torch.empty(max(K, 1), dtype=torch.int32, device=dev)
    gs = torch.empty(max(K, 1), dtype=torch.int32, device=dev)
    e1 = C.c_int64(0)
    _lib.check(L.dg_debug_sorted_instances(C.byref(a), out[5].data_ptr(), out[6].data_ptr(), _lib.ptr(out[8]),
                                           out[7].data_ptr(), int(out[0]), int(out[1]), tiles.data_ptr(),
                                           gs.data_ptr(),
                                           C.byref(e1), _lib.stream_of(dev)))
    torch.cuda.synchronize()
    return tiles[:K].cpu().numpy().view(np.uint32), gs[:K].cpu().numpy().view(np.uint32), int(e1.value)


def per_tile_lists(tiles, gids, e1):
    """tile -> list of Gaussians: the tile's phase-1 entries followed by its phase-2 entries."""
    lists = {}
    for part in (slice(0, e1), slice(e1, len(tiles))):
        for t, g in zip(tiles[part].tolist(), gids[part].tolist()):
            lists.setdefault(t, []).append(g)
    return lists


def hip_geometry(out, P, dev):
    from dogs_amd import _lib
    xy = torch.empty((P, 2), device=dev)
    co = torch.empty((P, 4), device=dev)
    rgbi = torch.empty((P, 4), device=dev)
    cnt = torch.empty(P, dtype=torch.int32, device=dev)
    _lib.check(_lib.load().dg_debug_geometry(out[5].data_ptr(), P, xy.data_ptr(), co.data_ptr(), rgbi.data_ptr(),
                                             cnt.data_ptr(), _lib.stream_of(dev)))
    torch.cuda.synchronize()
    return xy.cpu().numpy(), co.cpu().numpy(), rgbi.cpu().numpy(), cnt.cpu().numpy().view(np.uint32)


def hip_image_state(out, W, H, dev):
    from dogs_amd import _lib
    T = ((W + 15) // 16) * ((H + 15) // 16)
    fT = torch.empty(H * W, device=dev)
    nc = torch.empty(H * W, dtype=torch.int32, device=dev)
    mc = torch.empty(T, dtype=torch.int32, device=dev)
    rg = torch.empty((T, 2), dtype=torch.int32, device=dev)
    _lib.check(_lib.load().dg_debug_image_state(out[7].data_ptr(), W, H, fT.data_ptr(), nc.data_ptr(), mc.data_ptr(),
                                                rg.data_ptr(), _lib.stream_of(dev)))
    torch.cuda.synchronize()
    return (fT.cpu().numpy().reshape(H, W), nc.cpu().numpy().view(np.uint32).reshape(H, W),
            mc.cpu().numpy().view(np.uint32), rg.cpu().numpy().view(np.uint32))


def psnr(a, b):
    mse = float(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2))
    return float("inf") if mse == 0 else -10.0 * np.log10(mse)


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    n = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / (n if n > 0 else 1.0))


def yaw_view(s, yaw_deg, fx=1600.0):
    """The scene seen by a camera at the origin rotated about +y by yaw_deg (dogs_amd.camera.yaw_world_to_camera):
    the seeded view batches of SURVEY.md §8(d)."""
    import dataclasses
    import math
    from dogs_amd.camera import make_camera, yaw_world_to_camera
    c = s.camera
    cam = make_camera(c.width, c.height, fx, fx, world_to_camera=yaw_world_to_camera(math.radians(yaw_deg)))
    return dataclasses.replace(s, camera=cam)


def check_binned_prefix(t_h, i_h, e1, t_o, i_o, ranges_o, max_contrib):
    """Vectorised form of the per-tile prefix check: every tile's binned list (its phase-1 entries, then its phase-2
    entries) equals the first entries of the reference's (tile, depth bits, index) list, and reaches the tile's last
    contributor.  Returns (max binned list length, number of tiles with a phase-2 list)."""
    t_h = np.asarray(t_h, np.int64)
    i_h = np.asarray(i_h, np.int64)
    order = np.argsort(t_h, kind="stable")          # phase-1 entries stay ahead of phase-2 ones within a tile
    ts, gs = t_h[order], i_h[order]
    first = np.searchsorted(ts, ts, side="left")
    rank = np.arange(len(ts)) - first
    r0 = ranges_o[:, 0].astype(np.int64)
    rlen = (ranges_o[:, 1].astype(np.int64) - r0)
    assert (rank < rlen[ts]).all(), "a tile's binned list is longer than the reference list"
    bad = np.nonzero(np.asarray(i_o, np.int64)[r0[ts] + rank] != gs)[0]
    assert len(bad) == 0, f"{len(bad)} binned entries differ from the reference order (first tile {ts[bad[0]]})"
    T = len(ranges_o)
    cnt = np.bincount(ts, minlength=T)
    short = np.nonzero(np.asarray(max_contrib, np.int64) > cnt)[0]
    assert len(short) == 0, f"tile {short[:5]}: max contributor beyond the binned list"
    p2 = np.unique(t_h[e1:]) if len(t_h) > e1 else np.zeros(0)
    return int(cnt.max()) if T else 0, int(len(p2))
