"""numpy restatement of the reference's export paths -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/.  The product path (dogs_amd/export.py -> dg_splat_pack / dg_ply_pack) must never import it.

Follows conerf/model/gaussian_fields/gaussian_splat_model.py save_ply (:616-640) and save_splat (:666-708) op by op,
with numpy float32 scalars as the reference's loop sees them; the PLY element is built with the reference's own
structured-array assignment (so numpy's float -> u1 cast is the reference's).  plyfile is not installed here: the
header is the one plyfile writes for this element (format binary_little_endian 1.0, 'float' for f4, 'uchar' for
u1).  Parity unpinned: the reference ships no fixture for these writers.
"""
from __future__ import annotations

import numpy as np

SH_C0 = 0.28209479177387814  # sh_utils.py:26
FIELDS = [("x", "f4"), ("y", "f4"), ("z", "f4"), ("nx", "f4"), ("ny", "f4"), ("nz", "f4"),
          ("red", "u1"), ("green", "u1"), ("blue", "u1")]


def ply_header(n: int) -> bytes:
    names = {"f4": "float", "u1": "uchar"}
    lines = ["ply", "format binary_little_endian 1.0", f"element vertex {n}"]
    lines += [f"property {names[t]} {f}" for f, t in FIELDS] + ["end_header"]
    return ("\n".join(lines) + "\n").encode("ascii")


def ply_body(xyz: np.ndarray, f_dc: np.ndarray) -> bytes:
    """save_ply: rgbs = clamp_min(C0 * dc + 0.5, 0) * 255 (torch float32, then numpy float32 * 255)."""
    xyz = np.asarray(xyz, np.float32)
    dc = np.asarray(f_dc, np.float32).reshape(-1, 3)
    sh2rgb = (np.float32(SH_C0) * dc).astype(np.float32)
    rgbs = np.maximum(sh2rgb + np.float32(0.5), np.float32(0.0)).astype(np.float32) * 255
    normals = np.zeros_like(xyz)
    elements = np.empty(xyz.shape[0], dtype=FIELDS)
    attributes = np.concatenate((xyz, normals, rgbs), axis=1)
    # `elements[:] = list(map(tuple, attributes))` in the reference's numpy 1.x casts the float32 colour to u1 as
    # C does on x86 (float -> int32 -> low byte: 300.0 -> 44); numpy 2 raises instead, so the cast is spelled out
    for k, (f, t) in enumerate(FIELDS):
        col = attributes[:, k]
        elements[f] = col if t == "f4" else (col.astype(np.int64) & 0xFF).astype(np.uint8)
    return elements.tobytes()


def splat_body(xyz, scaling, opacity, rotation, f_dc) -> bytes:
    """save_splat, the reference's loop over argsort(-exp(s0 + s1 + s2) / (1 + exp(o)))."""
    xyz = np.asarray(xyz, np.float32).reshape(-1, 3)
    scale = np.asarray(scaling, np.float32).reshape(-1, 3)
    opacity = np.asarray(opacity, np.float32).reshape(-1, 1)
    quaternion = np.asarray(rotation, np.float32).reshape(-1, 4)
    features_dc = np.asarray(f_dc, np.float32).reshape(-1, 3)
    sorted_indices = np.argsort(-np.exp(scale[:, 0] + scale[:, 1] + scale[:, 2]) / (1 + np.exp(opacity[:, 0])),
                                kind="stable")
    out = []
    for idx in sorted_indices:
        position = np.array([xyz[idx][0], xyz[idx][1], xyz[idx][2]], dtype=np.float32)
        scales = np.exp(np.array([scale[idx][0], scale[idx][1], scale[idx][2]], dtype=np.float32))
        rot = np.array([quaternion[idx][0], quaternion[idx][1], quaternion[idx][2], quaternion[idx][3]],
                       dtype=np.float32)
        color = np.array([0.5 + SH_C0 * features_dc[idx][0], 0.5 + SH_C0 * features_dc[idx][1],
                          0.5 + SH_C0 * features_dc[idx][2], 1 / (1 + np.exp(-opacity[idx, 0]))])
        out.append(position.tobytes())
        out.append(scales.tobytes())
        out.append((color * 255).clip(0, 255).astype(np.uint8).tobytes())
        out.append(((rot / np.linalg.norm(rot)) * 128 + 128).clip(0, 255).astype(np.uint8).tobytes())
    return b"".join(out)


def splat_records(body: bytes):
    """Parse a .splat body into (position [N,3] f32, scale [N,3] f32, rgba [N,4] u8, rot [N,4] u8)."""
    rec = np.frombuffer(body, dtype=[("p", "<f4", 3), ("s", "<f4", 3), ("c", "u1", 4), ("q", "u1", 4)])
    return rec["p"], rec["s"], rec["c"], rec["q"]


def bounding_box2d(points, scale_factor=(1.0, 1.0), hmin=-1.0, hmax=1.0, p0=0.02, p1=0.98):
    """conerf/datasets/utils.py:112-150 in float64 (the reference runs it on torch.from_numpy of float64 points)."""
    points = np.asarray(points, np.float64)
    n = points.shape[0]
    sp = np.sort(points, axis=0)
    P0, P1 = int(p0 * (n - 1)), int(p1 * (n - 1))
    A, B = np.array([sp[P0, 0], sp[P0, 1]]), np.array([sp[P1, 0], sp[P1, 1]])
    Cc = (A + B) / 2.0
    half = np.linalg.norm(B - A) / 2.0
    ca, cb = (A - Cc) / np.linalg.norm(A - Cc), (B - Cc) / np.linalg.norm(B - Cc)
    s = np.asarray(scale_factor, np.float64)
    A, B = Cc + ca * s * half, Cc + cb * s * half
    return np.concatenate([np.stack([A, B]), np.array([[hmin], [hmax]])], axis=-1)


def fuse_blocks(blocks, point_bboxes, T):
    """master_gaussian_trainer.py:37-100 on numpy: blocks = [dict(name -> array)], returns (fused dict, bboxes)."""
    T = np.asarray(T, np.float64)
    fused, boxes = {}, []
    for b, blk in enumerate(blocks):
        pts = np.asarray(blk["xyz"], np.float64)[:, :2]
        obb = pts @ T[:2, :2].T + T[:2, 2]            # trimesh.transform_points (affine)
        boxes.append(bounding_box2d(obb, [1.0, 1.0], -1.0, 1.0, 0.001, 0.999))
        A, B = np.asarray(point_bboxes[b]).reshape(2, 3)[0], np.asarray(point_bboxes[b]).reshape(2, 3)[1]
        keep = np.argwhere((A[0] <= obb[:, 0]) & (obb[:, 0] <= B[0]) &
                           (A[1] <= obb[:, 1]) & (obb[:, 1] <= B[1])).reshape(-1)
        for k, v in blk.items():
            fused.setdefault(k, []).append(np.asarray(v)[keep])
    return {k: np.concatenate(v, 0) for k, v in fused.items()}, boxes
