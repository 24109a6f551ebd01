"""Block fuse and export of the trained Gaussians, drop-in for the reference's functions:

* `save_splat(model, path)`  -- GaussianSplatModel.save_splat (gaussian_splat_model.py:666-708).  The reference
  builds the 32-B records one Gaussian at a time in a Python loop; here `dg_splat_pack` sorts and packs them on the
  GPU and the host writes one buffer.
* `save_ply(model, path)`    -- GaussianSplatModel.save_ply (gaussian_splat_model.py:616-640): binary
  little-endian PLY with x y z nx ny nz (float) red green blue (uchar), records packed by `dg_ply_pack`; the
  header is the one plyfile writes for that element.
* `fuse_block_gaussians(...)` -- master_gaussian_trainer.py:37-100: per block, drop the Gaussians outside the
  block's initial grid cell (in the oriented-bounding-box frame), re-estimate the cell from the survivors, save
  the block's PLY, then concatenate the blocks.  Runs on the GPU tensors (the reference moves every block to numpy).
* `compute_bounding_box2D`, `points_in_bbox2D`, `compute_rainbow_color`, `save_colmap_ply` -- the helpers it uses
  (conerf/datasets/utils.py:112-299).

The model is duck-typed as in dogs_amd.densify (`_xyz`, `_features_dc`, `_scaling`, `_opacity`, `_quaternion`,
`_features_rest`).
"""
from __future__ import annotations

import ctypes as C
import math
import os

import numpy as np
import torch

from . import _lib

PLY_FIELDS = ("x", "y", "z", "nx", "ny", "nz", "red", "green", "blue")


def ply_header(n: int) -> bytes:
    """The header plyfile writes for PlyElement.describe(elements, 'vertex') with save_ply's dtype."""
    lines = ["ply", "format binary_little_endian 1.0", f"element vertex {n}"]
    lines += [f"property float {f}" for f in PLY_FIELDS[:6]] + [f"property uchar {f}" for f in PLY_FIELDS[6:]]
    lines.append("end_header")
    return ("\n".join(lines) + "\n").encode("ascii")


def _f32(t: torch.Tensor) -> torch.Tensor:
    t = t.detach()
    return t.contiguous() if t.dtype == torch.float32 else t.float().contiguous()


def splat_bytes(model) -> np.ndarray:
    """The .splat file body (uint8 [N * 32]) of save_splat, packed on the GPU."""
    xyz = _f32(model._xyz)
    dev = xyz.device
    _lib.require_device(xyz, "_xyz")
    n = int(xyz.shape[0])
    out = torch.empty(max(32 * n, 1), dtype=torch.uint8, device=dev)
    sc, op, q = _f32(model._scaling), _f32(model._opacity), _f32(model._quaternion)
    dc = _f32(model._features_dc)
    arena = _lib.TensorArena(dev)
    with _lib.device_ctx(dev):
        _lib.check(_lib.load().dg_splat_pack(n, xyz.data_ptr(), sc.data_ptr(), op.data_ptr(), q.data_ptr(),
                                             dc.data_ptr(), out.data_ptr(), arena.fn, None, _lib.stream_of(dev)))
    return out[:32 * n].cpu().numpy()


def ply_bytes(model) -> np.ndarray:
    """The save_ply vertex records (uint8 [N * 27]), packed on the GPU."""
    xyz = _f32(model._xyz)
    dev = xyz.device
    _lib.require_device(xyz, "_xyz")
    n = int(xyz.shape[0])
    dc = _f32(model._features_dc)
    out = torch.empty(max(27 * n, 1), dtype=torch.uint8, device=dev)
    with _lib.device_ctx(dev):
        _lib.check(_lib.load().dg_ply_pack(n, xyz.data_ptr(), dc.data_ptr(), out.data_ptr(), _lib.stream_of(dev)))
    return out[:27 * n].cpu().numpy()


@torch.no_grad()
def save_splat(model, output_path: str = "") -> None:
    body = splat_bytes(model)
    with open(output_path, "wb") as f:
        f.write(body.tobytes())


@torch.no_grad()
def save_ply(model, path: str) -> None:
    n = int(model._xyz.shape[0])
    body = ply_bytes(model)
    with open(path, "wb") as f:
        f.write(ply_header(n))
        f.write(body.tobytes())


# ---- block fuse (master_gaussian_trainer.py:37-100) and its helpers (conerf/datasets/utils.py)

def compute_bounding_box2D(points: torch.Tensor, scale_factor=(1.2, 1.2), bbox_min_height=-1.0, bbox_max_height=1.0,
                           p0=0.02, p1=0.98) -> torch.Tensor:
    """utils.py:112-150: a percentile AABB of the 2D points, enlarged about its centre; [2, 3] (z = heights)."""
    num_points = points.shape[0]
    scale = torch.tensor(list(scale_factor), dtype=points.dtype, device=points.device)
    sorted_points, _ = torch.sort(points, dim=0)
    P0, P1 = int(p0 * (num_points - 1)), int(p1 * (num_points - 1))
    aabb = torch.stack([sorted_points[P0, 0], sorted_points[P0, 1], sorted_points[P1, 0], sorted_points[P1, 1]])
    A, B = aabb[:2], aabb[2:]
    Cc = (A + B) / 2.0
    half_diagonal_len = torch.linalg.norm(B - A) / 2.0
    ca = (A - Cc) / torch.linalg.norm(A - Cc)
    cb = (B - Cc) / torch.linalg.norm(B - Cc)
    A = Cc + ca * scale * half_diagonal_len
    B = Cc + cb * scale * half_diagonal_len
    box = torch.cat([A, B], dim=0).reshape(2, 2)
    heights = torch.tensor([[bbox_min_height], [bbox_max_height]], dtype=box.dtype, device=box.device)
    return torch.cat([box, heights], dim=-1)


def transform_points2d(points: torch.Tensor, matrix) -> torch.Tensor:
    """trimesh.transform_points for [N, 2] points and a 3x3 homogeneous matrix (affine: no divide)."""
    m = torch.as_tensor(np.asarray(matrix), dtype=torch.float64, device=points.device)
    p = points.to(torch.float64)
    return p @ m[:2, :2].T + m[:2, 2]


def points_in_bbox2D(points: torch.Tensor, bbox, transform_world_to_obb=None) -> torch.Tensor:
    """utils.py:186-205: indices of the points inside the (closed) box, optionally in the OBB frame."""
    box = torch.as_tensor(np.asarray(bbox), device=points.device)
    A, B = box[0, :], box[1, :]
    p = transform_points2d(points, transform_world_to_obb) if transform_world_to_obb is not None else points
    inside = (A[0] <= p[:, 0]) & (p[:, 0] <= B[0]) & (A[1] <= p[:, 1]) & (p[:, 1] <= B[1])
    return torch.nonzero(inside).reshape(-1)


def compute_rainbow_color(block_id: int, freq: float = 0.4) -> torch.Tensor:
    """utils.py:282-288."""
    color = torch.zeros(1, 3)
    color[0, 0] = math.sin(freq * block_id + 0) * 0.5 + 0.5
    color[0, 1] = math.sin(freq * block_id + 2) * 0.5 + 0.5
    color[0, 2] = math.sin(freq * block_id + 4) * 0.5 + 0.5
    color *= 255.0
    return color


def save_colmap_ply(xyz: torch.Tensor, rgb: torch.Tensor, path: str) -> None:
    """utils.py:228-240 (COLMAP points3D.txt layout), the same text, built in one join instead of a write per point."""
    n = xyz.shape[0]
    x, c = xyz.detach().cpu().tolist(), rgb.detach().cpu().tolist()
    head = ("# 3D point list with one line of data per point:\n"
            "#   POINT3D_ID, X, Y, Z, R, G, B, ERROR, TRACK[] as (IMAGE_ID, POINT2D_IDX)\n"
            f"# Number of points: {n}, mean track length: 0\n")
    body = "".join(f"{i} {p[0]} {p[1]} {p[2]} {q[0]} {q[1]} {q[2]} 0 \n" for i, (p, q) in enumerate(zip(x, c)))
    with open(path, "w") as f:
        f.write(head + body)


@torch.no_grad()
def fuse_block_gaussians(block_gaussians: dict, point_bboxes=None, world_to_obb_transform=None, test_dir: str = ""):
    """master_gaussian_trainer.py:37-100.  Returns (xyz, features_dc, features_rest, scaling, quaternion, opacity,
    densify_point_bboxes); writes fuse_points3D_{block}.ply per block and non_overlap_points3D.txt."""
    xyz, opacity, features_dc, features_rest, scaling, quaternion = [], [], [], [], [], []
    densify_point_bboxes = [None] * (len(point_bboxes) if point_bboxes is not None else len(block_gaussians))
    all_xyz, all_rgb = [], []
    for block_id, model in block_gaussians.items():
        if point_bboxes is not None:
            point_bbox = np.asarray(point_bboxes[block_id]).reshape(2, 3)
            pts = model._xyz.detach()
            obb2d = transform_points2d(pts[:, :2], world_to_obb_transform)
            # re-estimated after densification (computed in float64 on the OBB points, as the reference's numpy path)
            densify_point_bboxes[block_id] = compute_bounding_box2D(obb2d, [1.0, 1.0], -1.0, 1.0, 0.001, 0.999).cpu()
            valid = points_in_bbox2D(obb2d, point_bbox)
            for a in ("_xyz", "_features_dc", "_features_rest", "_scaling", "_quaternion", "_opacity"):
                setattr(model, a, getattr(model, a)[valid])   # extract_sub_gaussians (gaussian_splat_model.py:308)
        xyz.append(model._xyz)
        features_dc.append(model._features_dc)
        features_rest.append(model._features_rest)
        scaling.append(model._scaling)
        quaternion.append(model._quaternion)
        opacity.append(model._opacity)
        pts = model._xyz.detach().cpu()
        all_xyz.append(pts)
        all_rgb.append(compute_rainbow_color(block_id).reshape(1, -1).expand(pts.shape[0], -1))
        save_ply(model, os.path.join(test_dir, f"fuse_points3D_{block_id}.ply"))
    save_colmap_ply(torch.cat(all_xyz, 0), torch.cat(all_rgb, 0), os.path.join(test_dir, "non_overlap_points3D.txt"))
    return (torch.cat(xyz, 0), torch.cat(features_dc, 0), torch.cat(features_rest, 0), torch.cat(scaling, 0),
            torch.cat(quaternion, 0), torch.cat(opacity, 0), densify_point_bboxes)
