"""Golden vectors of the reference's scene normalisation (conerf/datasets/load_colmap.py:501-660): the reference's own
similarity_from_cameras, get_center and normalize_poses are taken from its source file by name (ast; the module
itself imports imageio / trimesh / pycolmap, absent here) and run on a small seeded camera rig and point cloud, in
this container only.  The outputs are frozen into tests/golden/normalize_expected.npz, which tests/test_normalize.py
checks dogs_amd/normalize.py against.

up_est_method="ground" calls pyransac3d (third-party, not installed): the module is provided by
dogs_amd.normalize.ransac_plane (the restatement of its published Plane.fit), so the code around the plane fit is
pinned, the fit itself is not.  up_est_method="camera" raises in the reference (a [N,4] minus [3] broadcast); the
fixture records that.

usage: python tests/golden/make_normalize_golden.py   (from the repo root, where /root/reference exists)"""
import ast
import math
import os
import random
import sys
import types

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
SRC = "/root/reference/conerf/datasets/load_colmap.py"


def reference_functions():
    tree = ast.parse(open(SRC).read())
    keep = [n for n in tree.body if isinstance(n, ast.FunctionDef) and
            n.name in ("similarity_from_cameras", "get_center", "normalize_poses")]
    ns = {"np": np, "torch": torch, "F": F, "random": random, "math": math}
    exec(compile(ast.Module(body=keep, type_ignores=[]), SRC, "exec"), ns)
    return ns


def rig(seed=0, n_cams=24, n_pts=3000):
    """Cameras on a noisy ring looking at the origin (OpenCV c2w, y down), points on a tilted ground plane plus
    clutter above it."""
    g = np.random.default_rng(seed)
    c2w = []
    for k in range(n_cams):
        a = 2 * math.pi * k / n_cams
        pos = np.array([4 * math.cos(a), 4 * math.sin(a), 1.5]) + g.normal(0, 0.1, 3)
        fwd = -pos / np.linalg.norm(pos)
        up = np.array([0.0, 0.0, 1.0])
        right = np.cross(fwd, up); right /= np.linalg.norm(right)
        down = np.cross(fwd, right)
        M = np.eye(4)
        M[:3, 0], M[:3, 1], M[:3, 2], M[:3, 3] = right, down, fwd, pos
        c2w.append(M)
    tilt = np.array([[1, 0, 0], [0, math.cos(0.2), -math.sin(0.2)], [0, math.sin(0.2), math.cos(0.2)]])
    ground = np.concatenate([g.uniform(-3, 3, (n_pts, 2)), g.normal(0, 0.002, (n_pts, 1))], 1) @ tilt.T
    clutter = g.uniform(-1, 1, (n_pts // 3, 3)) + np.array([0, 0, 0.8])
    return np.stack(c2w), np.concatenate([ground, clutter], 0)


def main():
    sys.path.insert(0, ROOT)
    from dogs_amd.normalize import ransac_plane
    ns = reference_functions()

    class Plane:
        def fit(self, pts, thresh=0.05, minPoints=100, maxIteration=1000):  # noqa: N803
            return ransac_plane(pts, thresh, maxIteration, device="cpu")

    sys.modules["pyransac3d"] = types.SimpleNamespace(Plane=Plane)
    c2w, pts = rig()
    out = {"c2w": c2w, "pts": pts}
    for strict in (False, True):
        T, s = ns["similarity_from_cameras"](c2w, strict_scaling=strict)
        out[f"sim_T_{int(strict)}"], out[f"sim_s_{int(strict)}"] = T, np.array(s)
    T, s = ns["similarity_from_cameras"](c2w, strict_scaling=False)
    cw = np.einsum("nij, ki -> nkj", c2w, T)
    cw[:, :3, 3:4] *= s
    p = s * (T[:3, :3] @ pts.T + T[:3, 3][..., None]).T
    try:   # up_est_method="camera" raises in the reference itself ([N,4] poses[..., 3] minus a [3] centre)
        ns["normalize_poses"](torch.from_numpy(cw).float(), torch.from_numpy(p).float(), up_est_method="camera")
        out["camera_up_raises"] = np.array(False)
    except RuntimeError:
        out["camera_up_raises"] = np.array(True)
    for up, center in (("ground", "lookat"), ("ground", "camera"), ("ground", "point")):
        poses, pp, R, t = ns["normalize_poses"](torch.from_numpy(cw).float(), torch.from_numpy(p).float(),
                                                up_est_method=up, center_est_method=center)
        key = f"{up}_{center}"
        out[f"poses_{key}"], out[f"pts_{key}"] = poses.numpy(), pp.numpy()
        out[f"R_{key}"], out[f"t_{key}"] = R.numpy(), t.numpy()
    np.savez_compressed(os.path.join(HERE, "normalize_expected.npz"), **out)
    print("wrote", os.path.join(HERE, "normalize_expected.npz"), sorted(out))


if __name__ == "__main__":
    main()
