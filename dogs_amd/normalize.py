"""Scene normalisation before the block split (conerf/datasets/load_colmap.py:294-313): the COLMAP poses and points are
moved into the frame the reference clusters blocks in.

* `similarity_from_cameras(c2w, strict_scaling)` -- load_colmap.py:501-560 (after nerf-factory): rotate the mean
  camera "up" (-y in camera space) onto +z, recentre on the median of the cameras' nearest points to the origin along
  their view rays, scale by 1 / median (or max) camera distance.  numpy float64, operation for operation.
* `normalize_poses(poses, pts, up_est_method, center_est_method)` -- :573-660: the scene centre from the camera rays
  ("lookat": least squares between each camera's ray and its predecessor's), the up axis from the ground plane
  ("ground": RANSAC plane of the points, pyransac3d.Plane.fit(pts, thresh=0.01) with random.seed(0)) or from the
  cameras ("camera"); then rotation + translation of poses and points.  torch float32 as the reference.
* `normalize_scene(camtoworlds, points3d, scale, rotate)` -- the two in load_colmap's order (:294-313).

pyransac3d is a third-party dependency (scripts/env/install.sh:13, unpinned) that is absent here: `ransac_plane`
restates its published Plane.fit (for each of maxIteration iterations: random.sample 3 point indices, plane through
them with the unit normal cross(p1 - p0, p2 - p0), inliers |n.p + k| / |n| <= thresh, keep the first plane with the
most inliers), the candidate planes' inlier counts evaluated on the device in batches with the float32 operation order
of its numpy expression.  The plane fit is therefore parity-unpinned; the rest is pinned by golden vectors the
reference's own functions produced (tests/golden/make_normalize_golden.py)."""
from __future__ import annotations

import random

import numpy as np
import torch
import torch.nn.functional as F


def similarity_from_cameras(c2w: np.ndarray, strict_scaling: bool):
    """load_colmap.py:501-560 -> (transform [4,4], scale)."""
    t = c2w[:, :3, 3]
    R = c2w[:, :3, :3]
    ups = np.sum(R * np.array([0, -1.0, 0]), axis=-1)
    world_up = np.mean(ups, axis=0)
    world_up /= np.linalg.norm(world_up)
    up_camspace = np.array([0.0, -1.0, 0.0])
    c = (up_camspace * world_up).sum()
    cross = np.cross(world_up, up_camspace)
    skew = np.array([[0.0, -cross[2], cross[1]], [cross[2], 0.0, -cross[0]], [-cross[1], cross[0], 0.0]])
    if c > -1:
        R_align = np.eye(3) + skew + (skew @ skew) * 1 / (1 + c)
    else:  # y+ up: rotate 180 degrees about x
        R_align = np.array([[-1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [0.0, 0.0, 1.0]])
    R = R_align @ R
    fwds = np.sum(R * np.array([0, 0.0, 1.0]), axis=-1)
    t = (R_align @ t[..., None])[..., 0]
    nearest = t + (fwds * -t).sum(-1)[:, None] * fwds
    translate = -np.median(nearest, axis=0)
    transform = np.eye(4)
    transform[:3, 3] = translate
    transform[:3, :3] = R_align
    scale_fn = np.max if strict_scaling else np.median
    scale = 1.0 / scale_fn(np.linalg.norm(t + translate, axis=-1))
    return transform, scale


def ransac_plane(pts: np.ndarray, thresh: float = 0.05, max_iteration: int = 1000, batch: int = 64,
                 device=None):
    """pyransac3d.Plane.fit(pts, thresh, maxIteration) (published algorithm, see the module docstring): the sample
    indices come from Python's `random` in the same call sequence, so the caller's random.seed(0) fixes them."""
    pts = np.asarray(pts)
    n = pts.shape[0]
    samples = [random.sample(range(0, n), 3) for _ in range(max_iteration)]
    eqs = []
    for ids in samples:
        p = pts[ids]
        vec_a = p[1, :] - p[0, :]
        vec_b = p[2, :] - p[0, :]
        vec_c = np.cross(vec_a, vec_b)
        vec_c = vec_c / np.linalg.norm(vec_c)
        k = -np.sum(np.multiply(vec_c, p[1, :]))
        eqs.append([vec_c[0], vec_c[1], vec_c[2], k])
    eq = np.array(eqs, dtype=pts.dtype)
    norm = np.sqrt(eq[:, 0] ** 2 + eq[:, 1] ** 2 + eq[:, 2] ** 2).astype(pts.dtype)
    dev = torch.device(device) if device is not None else (
        torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
    P = torch.as_tensor(pts, device=dev)
    x, y, z = P[:, 0], P[:, 1], P[:, 2]
    counts = []
    for b0 in range(0, max_iteration, batch):
        e = torch.as_tensor(eq[b0:b0 + batch], device=dev)
        nn_ = torch.as_tensor(norm[b0:b0 + batch], device=dev)
        # ((a x + b y) + c z) + d, then / |n|: numpy's elementwise order in the array dtype
        d = (((e[:, 0:1] * x[None] + e[:, 1:2] * y[None]) + e[:, 2:3] * z[None]) + e[:, 3:4]) / nn_[:, None]
        counts.append((d.abs() <= thresh).sum(dim=1).cpu())
    counts = torch.cat(counts).numpy()
    best = -1
    best_n = 0
    for i, c in enumerate(counts.tolist()):   # strictly more inliers replaces the best (the first maximum wins)
        if c > best_n:
            best, best_n = i, c
    if best < 0:
        return [], np.array([], dtype=np.int64)
    e = torch.as_tensor(eq[best], device=dev)
    d = (((e[0] * x + e[1] * y) + e[2] * z) + e[3]) / torch.as_tensor(norm[best], device=dev)
    inl = torch.nonzero(d.abs() <= thresh).squeeze(-1).cpu().numpy()
    return [eq[best][0], eq[best][1], eq[best][2], eq[best][3]], inl


def normalize_poses(poses: torch.Tensor, pts: torch.Tensor, up_est_method: str = "ground",
                    center_est_method: str = "lookat"):
    """load_colmap.py:573-660 -> (poses_norm, pts, R, t)."""
    if center_est_method == "camera":
        center = poses[..., :3, 3].mean(0)
    elif center_est_method == "lookat":
        cams_ori = poses[..., :3, 3]
        cams_dir = poses[:, :3, :3] @ torch.as_tensor([0., 0., -1.])
        cams_dir = F.normalize(cams_dir, dim=-1)
        A = torch.stack([cams_dir, -cams_dir.roll(1, 0)], dim=-1)
        b = -cams_ori + cams_ori.roll(1, 0)
        t = torch.linalg.lstsq(A, b).solution
        center = (torch.stack([cams_dir, cams_dir.roll(1, 0)], dim=-1) * t[:, None, :] +
                  torch.stack([cams_ori, cams_ori.roll(1, 0)], dim=-1)).mean((0, 2))
    elif center_est_method == "point":
        center = poses[..., :3, 3].mean(0)
    else:
        raise NotImplementedError(f"Unknown center estimation method: {center_est_method}")
    if up_est_method == "ground":
        random.seed(0)
        plane_eq = ransac_plane(pts.numpy(), thresh=0.01)[0]
        plane_eq = torch.as_tensor(np.array(plane_eq))
        z = F.normalize(plane_eq[:3], dim=-1)
        signed_distance = (torch.cat([pts, torch.ones_like(pts[..., 0:1])], dim=-1) * plane_eq).sum(-1)
        if signed_distance.mean() < 0:
            z = -z
    elif up_est_method == "camera":
        z = F.normalize((poses[..., 3] - center).mean(0), dim=0)
    else:
        raise NotImplementedError(f"Unknown up estimation method: {up_est_method}")
    y = torch.as_tensor([z[1], -z[0], 0.])
    x = F.normalize(y.cross(z, dim=0), dim=0)
    y = z.cross(x, dim=0)
    if center_est_method == "point":
        Rc = torch.stack([x, y, z], dim=1)
        R = Rc.T
        inv_trans = torch.cat([torch.cat([R, torch.as_tensor([[0., 0., 0.]]).T], dim=1),
                               torch.as_tensor([[0., 0., 0., 1.]])], dim=0)
        poses_norm = (inv_trans @ poses)[:, :3]
        pts = (inv_trans @ torch.cat([pts, torch.ones_like(pts[:, 0:1])], dim=-1)[..., None])[:, :3, 0]
        poses_min, poses_max = poses_norm[..., 3].min(0)[0], poses_norm[..., 3].max(0)[0]
        pts_fg = pts[(poses_min[0] < pts[:, 0]) & (pts[:, 0] < poses_max[0]) &
                     (poses_min[1] < pts[:, 1]) & (pts[:, 1] < poses_max[1])]
        center = get_center(pts_fg)
        t = -center.reshape(3, 1)
        inv_trans = torch.cat([torch.cat([torch.eye(3), t], dim=1), torch.as_tensor([[0., 0., 0., 1.]])], dim=0)
        poses_norm = inv_trans @ poses
    else:
        Rc = torch.stack([x, y, z], dim=1)
        tc = center.reshape(3, 1)
        R, t = Rc.T, -Rc.T @ tc
        inv_trans = torch.cat([torch.cat([R, t], dim=1), torch.as_tensor([[0., 0., 0., 1.]])], dim=0)
        poses_norm = inv_trans @ poses
        pts = (R @ pts.T + t).T
    return poses_norm, pts, R, t


def get_center(pts: torch.Tensor) -> torch.Tensor:
    """load_colmap.py:563-570."""
    center = pts.mean(0)
    dis = (pts - center[None, :]).norm(p=2, dim=-1)
    mean, std = dis.mean(), dis.std()
    q25, q75 = torch.quantile(dis, 0.25), torch.quantile(dis, 0.75)
    valid = (dis > mean - 1.5 * std) & (dis < mean + 1.5 * std) & \
            (dis > mean - (q75 - q25) * 1.5) & (dis < mean + (q75 - q25) * 1.5)
    return pts[valid].mean(0)


def normalize_scene(camtoworlds: np.ndarray, points3d: np.ndarray, scale: bool = True, rotate: bool = True,
                    up_est_method: str = "ground", center_est_method: str = "lookat"):
    """load_colmap.py:294-313 -> (camtoworlds, points3d)."""
    c2w, pts = np.asarray(camtoworlds), np.asarray(points3d)
    if scale:
        T, s = similarity_from_cameras(c2w, strict_scaling=False)
        c2w = np.einsum("nij, ki -> nkj", c2w, T)
        c2w[:, :3, 3:4] *= s
        pts = s * (T[:3, :3] @ pts.T + T[:3, 3][..., None]).T
        if rotate:
            poses, p3, _, _ = normalize_poses(torch.from_numpy(c2w).float(), torch.from_numpy(pts).float(),
                                              up_est_method=up_est_method, center_est_method=center_est_method)
            c2w, pts = poses.numpy(), p3
    return c2w, pts
