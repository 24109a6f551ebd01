"""CPU restatement of the reference's Grid2D block split -- TEST INFRASTRUCTURE ONLY (the checker of
dogs_amd/blocksplit.py and dg_points_in_boxes2d; never imported by the product path).

Follows, line by line:
  conerf/datasets/utils.py:64-83    expand_bounding_box
  conerf/datasets/utils.py:93-109   compute_bounding_box2D_trimesh (trimesh.bounds.oriented_bounds_2D restated below)
  conerf/datasets/utils.py:112-148  compute_bounding_box2D
  conerf/datasets/utils.py:186-206  points_in_bbox2D
  conerf/geometry/cluster.py:73-140 Grid2DXY
  conerf/geometry/cluster.py:143-199 Grid2DClustering

trimesh is not installed here (and not vendored in the reference): oriented_bounds_2D and transform_points are
restated from trimesh's published algorithm (convex hull with qhull 'QbB'; every hull edge direction tried; minimum
area; offset centres the box; a 90-degree flip puts the long side on x).  The reference has no test or fixture for
this code, so the whole split is PARITY UNPINNED: the restatement is checked by known-answer cases
(tests/test_oracle_blocksplit.py) and the GPU path against this restatement.

Numerical conventions (the product follows the same ones): f64 throughout; a frame transform is
(T00 x + T01 y) + T02 without contraction; vector norms are sqrt(dx*dx + dy*dy); scale factors are the float32
values torch.tensor(list) makes of them, promoted to f64; sin/cos/atan2 from Python's math module.
Scalar loops in plain Python on purpose (small inputs: the boxes, the hull)."""
from __future__ import annotations

import math

import numpy as np


def _f32(v: float) -> float:
    return float(np.float32(v))


def transform_points(points2d: np.ndarray, T: np.ndarray) -> np.ndarray:
    p = np.asarray(points2d, dtype=np.float64)
    x, y = p[:, 0], p[:, 1]
    return np.stack([(T[0, 0] * x + T[0, 1] * y) + T[0, 2], (T[1, 0] * x + T[1, 1] * y) + T[1, 2]], axis=1)


def points_in_bbox2D(points: np.ndarray, bbox: np.ndarray, transform_world_to_obb: np.ndarray | None = None):
    """utils.py:186-206: indices (ascending) of the points inside [A, B] (inclusive), optionally in the OBB frame."""
    p = np.asarray(points, dtype=np.float64)[:, :2]
    if transform_world_to_obb is not None:
        p = transform_points(p, transform_world_to_obb)
    A, B = bbox[0], bbox[1]
    inside = (A[0] <= p[:, 0]) & (p[:, 0] <= B[0]) & (A[1] <= p[:, 1]) & (p[:, 1] <= B[1])
    return np.nonzero(inside)[0].astype(np.int64)


def _diag_expand(ax, ay, bx, by, sx, sy):
    """The corner recomputation shared by utils.py:72-81 and :136-143: C +- dir * scale * half_diagonal."""
    cx, cy = (ax + bx) / 2.0, (ay + by) / 2.0
    half = math.sqrt((bx - ax) * (bx - ax) + (by - ay) * (by - ay)) / 2.0
    na = math.sqrt((ax - cx) * (ax - cx) + (ay - cy) * (ay - cy))
    nb = math.sqrt((bx - cx) * (bx - cx) + (by - cy) * (by - cy))
    dax, day = (ax - cx) / na, (ay - cy) / na
    dbx, dby = (bx - cx) / nb, (by - cy) / nb
    return (cx + dax * sx * half, cy + day * sy * half, cx + dbx * sx * half, cy + dby * sy * half)


def compute_bounding_box2D(points: np.ndarray, scale_factor=(1.2, 1.2), bbox_min_height=-1.0, bbox_max_height=1.0,
                           p0=0.02, p1=0.98) -> np.ndarray:
    """utils.py:112-148: per-column order statistics at int(p * (n - 1)), expanded along the diagonal -> [2, 3]."""
    p = np.asarray(points, dtype=np.float64)
    n = p.shape[0]
    sx = np.sort(p[:, 0])
    sy = np.sort(p[:, 1])
    i0, i1 = int(p0 * (n - 1)), int(p1 * (n - 1))
    ax, ay, bx, by = _diag_expand(float(sx[i0]), float(sy[i0]), float(sx[i1]), float(sy[i1]),
                                  _f32(scale_factor[0]), _f32(scale_factor[1]))
    return np.array([[ax, ay, _f32(bbox_min_height)], [bx, by, _f32(bbox_max_height)]], dtype=np.float64)


def expand_bounding_box(aabb4, scale_factor=(1.2, 1.2)) -> np.ndarray:
    """utils.py:64-83 for a 2D box [A0, A1, B0, B1] -> [2, 2]."""
    ax, ay, bx, by = (float(v) for v in aabb4)
    ax, ay, bx, by = _diag_expand(ax, ay, bx, by, _f32(scale_factor[0]), _f32(scale_factor[1]))
    return np.array([[ax, ay], [bx, by]], dtype=np.float64)


def _planar(ox: float, oy: float, theta: float) -> list:
    s, c = math.sin(theta), math.cos(theta)
    return [[c, s, ox], [-s, c, oy], [0.0, 0.0, 1.0]]


def oriented_bounds_2D(points: np.ndarray):
    """trimesh.bounds.oriented_bounds_2D: (3x3 world-to-OBB transform, extents [2]) of the minimum-area rectangle."""
    from scipy.spatial import ConvexHull
    pts = np.asarray(points, dtype=np.float64)
    hull = ConvexHull(pts, qhull_options="QbB")
    hull_pts = [(float(a), float(b)) for a, b in hull.points[hull.vertices]]
    best = None
    for i0, i1 in hull.simplices:
        ex = float(hull.points[i1, 0] - hull.points[i0, 0])
        ey = float(hull.points[i1, 1] - hull.points[i0, 1])
        nrm = math.sqrt(ex * ex + ey * ey)
        if not nrm > 1e-12:       # zero-length edges are skipped (trimesh unitize(check_valid=True))
            continue
        ex, ey = ex / nrm, ey / nrm
        px, py = -ey, ex
        xs = [ex * a + ey * b for a, b in hull_pts]
        ys = [px * a + py * b for a, b in hull_pts]
        b = (min(xs), min(ys), max(xs), max(ys))
        w, h = b[2] - b[0], b[3] - b[1]
        area = w * h
        if best is None or area < best[0]:
            best = (area, b, (w, h), (ex, ey))
    _, b, (w, h), (ex, ey) = best
    theta = math.atan2(ey, ex)
    T = _planar(-b[0] - w * 0.5, -b[1] - h * 0.5, theta)
    if w < h:
        F = _planar(0.0, 0.0, math.pi / 2)
        T = [[(F[r][0] * T[0][c] + F[r][1] * T[1][c]) + F[r][2] * T[2][c] for c in range(3)] for r in range(3)]
        w, h = h, w
    return np.array(T, dtype=np.float64), np.array([w, h], dtype=np.float64)


def compute_bounding_box2D_trimesh(points, bbox_min_height=-1.0, bbox_max_height=1.0, p0=0.02, p1=0.98):
    """utils.py:93-109: OBB of the points inside the loose percentile box."""
    aabb = compute_bounding_box2D(points, [1.0, 1.0], bbox_min_height, bbox_max_height, p0, p1)
    filtered = np.asarray(points, dtype=np.float64)[points_in_bbox2D(points, aabb)]
    T, extents = oriented_bounds_2D(filtered[:, :2])
    return extents, T


def Grid2DXY(points2d, bbox_min_height=-1.0, bbox_max_height=1.0, p0=0.02, p1=0.98, mx=1, my=1,
             use_prior_center=False, transform_world_to_obb=None):
    """cluster.py:73-140 -> (grid cells [2, 3] each, world-to-OBB transform)."""
    if transform_world_to_obb is None:
        _, transform_world_to_obb = compute_bounding_box2D_trimesh(points2d, bbox_min_height, bbox_max_height, p0, p1)
    obb = transform_points(np.asarray(points2d, dtype=np.float64)[:, :2], transform_world_to_obb)
    aabb = compute_bounding_box2D(obb, [1.0, 1.0], bbox_min_height, bbox_max_height, p0, p1)
    A, B = aabb[0], aabb[1]
    lo, hi = _f32(bbox_min_height), _f32(bbox_max_height)
    cells = []
    if use_prior_center and mx * my == 4:
        cells.append(np.array([[A[0], A[1], A[2]], [0.0, 0.0, hi]]))
        cells.append(np.array([[A[0], 0.0, lo], [0.0, B[1], hi]]))
        cells.append(np.array([[0.0, A[1], lo], [B[0], 0.0, hi]]))
        cells.append(np.array([[0.0, 0.0, lo], [B[0], B[1], B[2]]]))
        return cells, transform_world_to_obb
    xd = np.linspace(A[0], B[0], mx + 1)
    xcells = []
    for i in range(mx):
        box = np.array([[xd[i], A[1]], [xd[i + 1], B[1]]])
        inside = obb[points_in_bbox2D(obb, box)]
        xcells.append(compute_bounding_box2D(inside, [1.0, 1.0], bbox_min_height, bbox_max_height, 0, 1))
    for xc in xcells:
        yd = np.linspace(xc[0, 1], xc[1, 1], my + 1)
        for j in range(my):
            cells.append(np.array([[xc[0, 0], yd[j], lo], [xc[1, 0], yd[j + 1], hi]]))
    return cells, transform_world_to_obb


def Grid2DClustering(points, scale_factor=(1.2, 1.2), bbox_min_height=-1.0, bbox_max_height=1.0, p0=0.02, p1=0.98,
                     num_blocks=1, mx=1, my=1, use_prior_center=False, transform_world_to_obb=None):
    """cluster.py:143-199 -> (labels u8 [N], cells, expanded cells [2, 3] each, world-to-OBB transform)."""
    pts2 = np.asarray(points, dtype=np.float64)[:, :2]
    cells, T = Grid2DXY(pts2, bbox_min_height, bbox_max_height, p0, p1, mx, my, use_prior_center,
                        transform_world_to_obb)
    labels = np.zeros(pts2.shape[0], dtype=np.uint8)
    for k, cell in enumerate(cells):
        labels[points_in_bbox2D(pts2, cell, T)] = k
    lo, hi = _f32(bbox_min_height), _f32(bbox_max_height)
    exp_cells = []
    for cell in cells:
        e = expand_bounding_box(cell[:, :2].reshape(-1), scale_factor)
        exp_cells.append(np.concatenate([e, np.array([[lo], [hi]])], axis=1))
    return labels, cells, exp_cells, T
