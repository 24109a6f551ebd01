"""Grid2D block split of a scene, drop-in for the reference's functions:

* `cluster_image_in_grid(...)`  -- load_colmap.py:98-138: camera centres -> Grid2D cells, cluster.txt, and the
  images of each expanded cell.
* `cluster_points_in_grid(...)` -- load_colmap.py:141-177: the COLMAP points of each expanded cell, written as
  points3D_{k}.ply (store_ply's format, utils.py:382-397).
* `Grid2DClustering`, `Grid2DXY` -- cluster.py:73-199.
* `points_in_bbox2D`, `compute_bounding_box2D`, `compute_bounding_box2D_trimesh`, `expand_bounding_box`,
  `oriented_bounds_2D` (trimesh.bounds.oriented_bounds_2D) -- utils.py:64-206.

Every per-point pass runs on the GPU through `dg_points_in_boxes2d` (blocksplit.hip): the frame transform, all box
tests, the labels and the ascending member lists in one streaming pass per box set, where the reference re-reads
the cloud once per box.  Order statistics use a device sort; only O(boxes) and O(hull) scalar geometry runs on the
host.  Numerical conventions (f64; (T00 x + T01 y) + T02; sqrt(dx*dx + dy*dy); float32 scale factors; math.sin/cos)
are listed in oracle/blocksplit_oracle.py, the CPU restatement the tests compare against.  trimesh is absent here,
so the OBB follows trimesh's published algorithm and the split is parity-unpinned against the reference itself.
"""
from __future__ import annotations

import ctypes as C
import math
import os

import numpy as np
import torch

from . import _lib


def _device(device=None) -> torch.device:
    if device is not None:
        return torch.device(device)
    if not torch.cuda.is_available():
        raise RuntimeError("dogs_amd.blocksplit needs a HIP device: libdogs_hip has no CPU path")
    return torch.device("cuda", torch.cuda.current_device())


def _points_f64(points, device) -> torch.Tensor:
    t = torch.as_tensor(np.asarray(points) if not isinstance(points, torch.Tensor) else points)
    return t.to(device=device, dtype=torch.float64).contiguous()


def _f32(v) -> float:
    return float(np.float32(v))


def points_in_boxes2d(points, boxes, transform_world_to_obb=None, labels: bool = False, transformed: bool = False,
                      members: bool = True, device=None) -> dict:
    """One dg_points_in_boxes2d pass over `points` ([N, >= 2], x y in the first two columns) for up to 64 boxes
    ([A0, A1, B0, B1] or [2, >= 2] each).  Returns counts (numpy u32 [C]) and, as asked: members (list of device
    int64 index tensors, ascending), labels (device u8 [N]: the last box containing the point, 0 if none) and
    transformed (device f64 [N, 2]: the points in the box frame)."""
    dev = _device(device)
    p = _points_f64(points, dev)
    if p.dim() != 2 or p.shape[1] < 2:
        raise RuntimeError(f"points must be [N, >=2], got {tuple(p.shape)}")
    n, stride = int(p.shape[0]), int(p.shape[1])
    bx = [np.asarray(b, dtype=np.float64) for b in boxes]
    if not 1 <= len(bx) <= _lib.DG_MAX_BOXES:
        raise RuntimeError(f"1..{_lib.DG_MAX_BOXES} boxes per pass, got {len(bx)}")
    s = _lib.DgBox2dSet()
    s.C = len(bx)
    if transform_world_to_obb is not None:
        T = np.asarray(transform_world_to_obb, dtype=np.float64)
        s.has_T = 1
        for q, v in enumerate((T[0, 0], T[0, 1], T[0, 2], T[1, 0], T[1, 1], T[1, 2])):
            s.T[q] = float(v)
    for k, b in enumerate(bx):
        a0, a1, b0, b1 = (b[0], b[1], b[2], b[3]) if b.ndim == 1 else (b[0, 0], b[0, 1], b[1, 0], b[1, 1])
        for q, v in enumerate((a0, a1, b0, b1)):
            s.box[k][q] = float(v)
    lab = torch.empty(max(n, 1), dtype=torch.uint8, device=dev) if labels else None
    tra = torch.empty((max(n, 1), 2), dtype=torch.float64, device=dev) if transformed else None
    counts = (C.c_uint32 * len(bx))()
    arena = _lib.TensorArena(dev)
    with _lib.device_ctx(dev):
        _lib.check(_lib.load().dg_points_in_boxes2d(n, p.data_ptr() if n else None, stride, C.byref(s),
                                                    lab.data_ptr() if lab is not None else None,
                                                    tra.data_ptr() if tra is not None else None, counts,
                                                    1 if members else 0, arena.fn, None, _lib.stream_of(dev)))
    out = {"counts": np.array(counts[:], dtype=np.uint32)}
    if members:
        flat = arena.get(_lib.DG_BUF_MEMBERS)[: 4 * int(out["counts"].sum())].view(torch.int32)
        lists, o = [], 0
        for c in out["counts"].tolist():
            # u32 indices < 2^31 (N fits the u32 ABI; point clouds stay far below 2^31)
            lists.append(flat[o:o + c].to(torch.int64))
            o += c
        out["members"] = lists
    if labels:
        out["labels"] = lab[:n]
    if transformed:
        out["transformed"] = tra[:n]
    return out


def points_in_bbox2D(points, bbox, transform_world_to_obb=None) -> np.ndarray:
    """utils.py:186-206: ascending indices (int64) of the points inside the closed box, optionally in the OBB frame."""
    r = points_in_boxes2d(points, [np.asarray(bbox, dtype=np.float64)[:2, :2]], transform_world_to_obb)
    return r["members"][0].cpu().numpy()


def _diag_expand(ax, ay, bx, by, sx, sy):
    cx, cy = (ax + bx) / 2.0, (ay + by) / 2.0
    half = math.sqrt((bx - ax) * (bx - ax) + (by - ay) * (by - ay)) / 2.0
    na = math.sqrt((ax - cx) * (ax - cx) + (ay - cy) * (ay - cy))
    nb = math.sqrt((bx - cx) * (bx - cx) + (by - cy) * (by - cy))
    return (cx + (ax - cx) / na * sx * half, cy + (ay - cy) / na * sy * half,
            cx + (bx - cx) / nb * sx * half, cy + (by - cy) / nb * sy * half)


def _order_stats(p: torch.Tensor, p0: float, p1: float):
    n = int(p.shape[0])
    i0, i1 = int(p0 * (n - 1)), int(p1 * (n - 1))
    if i0 == 0 and i1 == n - 1:   # the extremes: a reduction gives the same elements as a sort
        lo, hi = p[:, :2].amin(dim=0), p[:, :2].amax(dim=0)
        v = torch.stack([lo[0], lo[1], hi[0], hi[1]]).cpu().tolist()
    else:
        srt, _ = torch.sort(p[:, :2], dim=0)
        v = torch.stack([srt[i0, 0], srt[i0, 1], srt[i1, 0], srt[i1, 1]]).cpu().tolist()
    return v


def compute_bounding_box2D(points, scale_factor=(1.2, 1.2), bbox_min_height=-1.0, bbox_max_height=1.0, p0=0.02,
                           p1=0.98, device=None) -> np.ndarray:
    """utils.py:112-148: the per-column order statistics at int(p * (n - 1)) (device sort), enlarged about the
    centre along the diagonal; [2, 3] with the heights in z."""
    p = _points_f64(points, _device(device))
    ax, ay, bx, by = _order_stats(p, p0, p1)
    ax, ay, bx, by = _diag_expand(ax, ay, bx, by, _f32(scale_factor[0]), _f32(scale_factor[1]))
    return np.array([[ax, ay, _f32(bbox_min_height)], [bx, by, _f32(bbox_max_height)]], dtype=np.float64)


def expand_bounding_box(aabb, scale_factor=(1.2, 1.2)) -> np.ndarray:
    """utils.py:64-83 for a 2D box [A0, A1, B0, B1] -> [2, 2]."""
    ax, ay, bx, by = (float(v) for v in np.asarray(aabb, dtype=np.float64).reshape(-1)[:4])
    return np.array(_diag_expand(ax, ay, bx, by, _f32(scale_factor[0]), _f32(scale_factor[1])),
                    dtype=np.float64).reshape(2, 2)


def _planar(ox: float, oy: float, theta: float) -> np.ndarray:
    s, c = math.sin(theta), math.cos(theta)
    return np.array([[c, s, ox], [-s, c, oy], [0.0, 0.0, 1.0]], dtype=np.float64)


def oriented_bounds_2D(points) -> tuple[np.ndarray, np.ndarray]:
    """trimesh.bounds.oriented_bounds_2D: the minimum-area rectangle over the convex hull's edge directions ->
    (3x3 world-to-OBB transform centring it with its long side on x, extents [2])."""
    from scipy.spatial import ConvexHull
    pts = np.asarray(points, dtype=np.float64)[:, :2]
    hull = ConvexHull(pts, qhull_options="QbB")
    hp = hull.points[hull.vertices]
    e = hull.points[hull.simplices[:, 1]] - hull.points[hull.simplices[:, 0]]
    nrm = np.sqrt(e[:, 0] * e[:, 0] + e[:, 1] * e[:, 1])
    ok = nrm > 1e-12
    e = e[ok] / nrm[ok, None]
    xs = e[:, :1] * hp[None, :, 0] + e[:, 1:] * hp[None, :, 1]        # [edges, hull points]
    ys = -e[:, 1:] * hp[None, :, 0] + e[:, :1] * hp[None, :, 1]
    b = np.stack([xs.min(1), ys.min(1), xs.max(1), ys.max(1)], axis=1)
    w, h = b[:, 2] - b[:, 0], b[:, 3] - b[:, 1]
    k = int(np.argmin(w * h))
    wk, hk = float(w[k]), float(h[k])
    T = _planar(-float(b[k, 0]) - wk * 0.5, -float(b[k, 1]) - hk * 0.5, math.atan2(float(e[k, 1]), float(e[k, 0])))
    if wk < hk:
        F = _planar(0.0, 0.0, math.pi / 2)
        T = np.array([[(F[r, 0] * T[0, c] + F[r, 1] * T[1, c]) + F[r, 2] * T[2, c] for c in range(3)]
                      for r in range(3)])
        wk, hk = hk, wk
    return T, np.array([wk, hk], dtype=np.float64)


def compute_bounding_box2D_trimesh(points, bbox_min_height=-1.0, bbox_max_height=1.0, p0=0.02, p1=0.98):
    """utils.py:93-109: (extents, world-to-OBB transform) of the points inside the loose percentile box."""
    dev = _device()
    p = _points_f64(points, dev)
    aabb = compute_bounding_box2D(p, [1.0, 1.0], bbox_min_height, bbox_max_height, p0, p1, device=dev)
    inside = points_in_boxes2d(p, [aabb[:, :2]], device=dev)["members"][0]
    T, extents = oriented_bounds_2D(p[inside, :2].cpu().numpy())
    return extents, T


def Grid2DXY(points2d, bbox_min_height=-1.0, bbox_max_height=1.0, p0=0.02, p1=0.98, mx=1, my=1,
             use_prior_center=False, transform_world_to_obb=None):
    """cluster.py:73-140 -> (grid cells [2, 3] each, world-to-OBB transform)."""
    dev = _device()
    p = _points_f64(points2d, dev)
    if transform_world_to_obb is None:
        _, transform_world_to_obb = compute_bounding_box2D_trimesh(p, bbox_min_height, bbox_max_height, p0, p1)
    everything = [np.array([-np.inf, -np.inf, np.inf, np.inf])]
    obb = points_in_boxes2d(p, everything, transform_world_to_obb, transformed=True, members=False,
                            device=dev)["transformed"]
    aabb = compute_bounding_box2D(obb, [1.0, 1.0], bbox_min_height, bbox_max_height, p0, p1, device=dev)
    A, B = aabb[0], aabb[1]
    lo, hi = _f32(bbox_min_height), _f32(bbox_max_height)
    if use_prior_center and mx * my == 4:
        cells = [np.array([[A[0], A[1], A[2]], [0.0, 0.0, hi]]), np.array([[A[0], 0.0, lo], [0.0, B[1], hi]]),
                 np.array([[0.0, A[1], lo], [B[0], 0.0, hi]]), np.array([[0.0, 0.0, lo], [B[0], B[1], B[2]]])]
        return cells, transform_world_to_obb
    xd = np.linspace(A[0], B[0], mx + 1)
    xboxes = [np.array([xd[i], A[1], xd[i + 1], B[1]]) for i in range(mx)]
    xcells = []
    for c0 in range(0, mx, _lib.DG_MAX_BOXES):   # all x-divisions in one pass per 64
        mem = points_in_boxes2d(obb, xboxes[c0:c0 + _lib.DG_MAX_BOXES], device=dev)["members"]
        for idx in mem:
            if idx.numel() == 0:
                raise IndexError("Grid2DXY: an x-division holds no points")
            xcells.append(compute_bounding_box2D(obb[idx], [1.0, 1.0], bbox_min_height, bbox_max_height, 0, 1,
                                                 device=dev))
    cells = []
    for xc in xcells:
        yd = np.linspace(xc[0, 1], xc[1, 1], my + 1)
        for j in range(my):
            cells.append(np.array([[xc[0, 0], yd[j], lo], [xc[1, 0], yd[j + 1], hi]]))
    return cells, transform_world_to_obb


def Grid2DClustering(points, scale_factor=(1.2, 1.2), bbox_min_height=-1.0, bbox_max_height=1.0, p0=0.02, p1=0.98,
                     num_blocks=1, mx=1, my=1, use_prior_center=False, transform_world_to_obb=None):  # noqa: ARG001
    """cluster.py:143-199 -> (labels u8 [N] numpy, cells, expanded cells ([2, 3] each), world-to-OBB transform).
    Labels: the last cell containing the point (0 when none), from one device pass over all cells."""
    dev = _device()
    p = _points_f64(points, dev)
    cells, T = Grid2DXY(p, bbox_min_height, bbox_max_height, p0, p1, mx, my, use_prior_center,
                        transform_world_to_obb)
    if len(cells) > _lib.DG_MAX_BOXES:
        raise RuntimeError(f"Grid2DClustering: at most {_lib.DG_MAX_BOXES} cells (got {len(cells)})")
    r = points_in_boxes2d(p, [c[:, :2] for c in cells], T, labels=True, members=False, device=dev)
    lo, hi = _f32(bbox_min_height), _f32(bbox_max_height)
    exp_cells = [np.concatenate([expand_bounding_box(c[:, :2].reshape(-1), scale_factor), np.array([[lo], [hi]])],
                                axis=1) for c in cells]
    return r["labels"].cpu().numpy(), cells, exp_cells, T


def _members_per_box(points, boxes, T, dev):
    out = []
    for c0 in range(0, len(boxes), _lib.DG_MAX_BOXES):
        out += points_in_boxes2d(points, [b[:, :2] for b in boxes[c0:c0 + _lib.DG_MAX_BOXES]], T,
                                 device=dev)["members"]
    return out


def store_ply(path: str, xyz: np.ndarray, color: np.ndarray) -> None:
    """utils.py:382-397: binary little-endian PLY, x y z nx ny nz (float, normals 0) red green blue (uchar)."""
    xyz = np.asarray(xyz)
    n = xyz.shape[0]
    rec = np.zeros(n, dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("nx", "<f4"), ("ny", "<f4"), ("nz", "<f4"),
                             ("red", "u1"), ("green", "u1"), ("blue", "u1")])
    for i, f in enumerate(("x", "y", "z")):
        rec[f] = xyz[:, i]
    col = np.asarray(color)
    for i, f in enumerate(("red", "green", "blue")):
        rec[f] = col[:, i]
    head = ["ply", "format binary_little_endian 1.0", f"element vertex {n}"]
    head += [f"property float {f}" for f in ("x", "y", "z", "nx", "ny", "nz")]
    head += [f"property uchar {f}" for f in ("red", "green", "blue")] + ["end_header"]
    with open(path, "wb") as fh:
        fh.write(("\n".join(head) + "\n").encode("ascii"))
        fh.write(rec.tobytes())


def cluster_image_in_grid(camtoworlds, save_dir: str, all_image_indices, bbox_scale_factor, image_index_to_image_id,
                          num_blocks: int = 1, mx: int = 1, my: int = 1):
    """load_colmap.py:98-138 -> (block_image_ids {k: [indices]}, bboxes [C,2,3], exp_bboxes [C,2,3], transform).
    Writes save_dir/cluster.txt ("image_id label" per image)."""
    dev = _device()
    centres = np.asarray(camtoworlds)[..., :3, -1]
    labels, bboxes, exp_bboxes, T = Grid2DClustering(centres, num_blocks=num_blocks, scale_factor=bbox_scale_factor[:2],
                                                     p0=0, p1=1, mx=mx, my=my)
    with open(os.path.join(save_dir, "cluster.txt"), "w", encoding="utf-8") as fh:
        for i, lab in enumerate(labels.tolist()):
            print(f"{image_index_to_image_id[i]} {lab}", file=fh)
    idx = np.asarray(all_image_indices)
    mem = _members_per_box(_points_f64(centres[:, :2], dev), exp_bboxes, T, dev)
    block_image_ids = {k: [idx[m.cpu().numpy()]] for k, m in enumerate(mem)}
    return block_image_ids, np.stack(bboxes, axis=0), np.stack(exp_bboxes, axis=0), T


def cluster_points_in_grid(points3d, colors, save_dir: str, bbox_scale_factor, num_blocks: int = 1, mx: int = 1,
                           my: int = 1, use_prior_center: bool = False, transform_world_to_obb=None):
    """load_colmap.py:141-177 -> (bboxes, exp_bboxes, transform).  Writes save_dir/points3D_{k}.ply for the points
    of each expanded cell (only when the file does not exist yet, as the reference)."""
    dev = _device()
    p = _points_f64(points3d, dev)
    _, bboxes, exp_bboxes, T = Grid2DClustering(p, num_blocks=num_blocks, scale_factor=bbox_scale_factor[:2],
                                                p0=0.00001, p1=0.99999, mx=mx, my=my,
                                                use_prior_center=use_prior_center,
                                                transform_world_to_obb=transform_world_to_obb)
    mem = _members_per_box(p, exp_bboxes, T, dev)
    pts_np, col_np = np.asarray(points3d), np.asarray(colors)
    for k, m in enumerate(mem):
        path = os.path.join(save_dir, f"points3D_{k}.ply")
        if not os.path.exists(path):
            sel = m.cpu().numpy()
            store_ply(path, pts_np[sel], col_np[sel])
    return np.stack(bboxes, axis=0), np.stack(exp_bboxes, axis=0), T
