"""Scene normalisation (dogs_amd/normalize.py, load_colmap.py:294-313, 501-660) against golden vectors produced by the
reference's own functions (tests/golden/make_normalize_golden.py): similarity_from_cameras bit for bit (numpy
float64, same operations), normalize_poses' poses / points / R / t for the three centre estimates with the ground-
plane up axis (the plane fit itself is the pyransac3d restatement in both, see the generator), the reference's own
failure of up_est_method="camera", and the RANSAC restatement's behaviour on a clean plane."""
import os
import random

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(os.path.join(HERE, "golden", "normalize_expected.npz")))


def test_similarity_from_cameras(gold):
    from dogs_amd.normalize import similarity_from_cameras
    for strict in (0, 1):
        T, s = similarity_from_cameras(gold["c2w"], strict_scaling=bool(strict))
        np.testing.assert_array_equal(T, gold[f"sim_T_{strict}"])
        assert s == float(gold[f"sim_s_{strict}"])


def test_normalize_poses(gold):
    from dogs_amd.normalize import normalize_poses, similarity_from_cameras
    T, s = similarity_from_cameras(gold["c2w"], strict_scaling=False)
    cw = np.einsum("nij, ki -> nkj", gold["c2w"], T)
    cw[:, :3, 3:4] *= s
    p = s * (T[:3, :3] @ gold["pts"].T + T[:3, 3][..., None]).T
    for center in ("lookat", "camera", "point"):
        poses, pp, R, t = normalize_poses(torch.from_numpy(cw).float(), torch.from_numpy(p).float(), "ground", center)
        k = f"ground_{center}"
        np.testing.assert_allclose(poses.numpy(), gold[f"poses_{k}"], rtol=0, atol=1e-6)
        np.testing.assert_allclose(pp.numpy(), gold[f"pts_{k}"], rtol=0, atol=1e-6)
        np.testing.assert_allclose(R.numpy(), gold[f"R_{k}"], rtol=0, atol=1e-6)
        np.testing.assert_allclose(t.numpy(), gold[f"t_{k}"], rtol=0, atol=1e-6)
    assert bool(gold["camera_up_raises"])
    with pytest.raises(RuntimeError):
        normalize_poses(torch.from_numpy(cw).float(), torch.from_numpy(p).float(), "camera", "lookat")


def test_ransac_plane_recovers_a_plane():
    from dogs_amd.normalize import ransac_plane
    g = np.random.default_rng(1)
    n = np.array([0.2, -0.3, 0.93]); n /= np.linalg.norm(n)
    pts = g.uniform(-2, 2, (4000, 3)).astype(np.float32)
    pts[:3000] -= (pts[:3000] @ n - 0.5)[:, None] * n[None].astype(np.float32)   # on the plane n.x = 0.5
    random.seed(0)
    eq, inl = ransac_plane(pts, thresh=0.01, device="cpu")
    nn = np.array(eq[:3], dtype=np.float64)
    assert abs(abs(nn @ n) - 1) < 1e-4 and len(inl) >= 3000
    random.seed(0)
    eq2, inl2 = ransac_plane(pts, thresh=0.01, batch=7, device="cpu")   # batching does not change the choice
    assert [float(x) for x in eq] == [float(x) for x in eq2] and np.array_equal(inl, inl2)


def test_normalize_scene_order(gold):
    from dogs_amd.normalize import normalize_scene
    c2w, pts = normalize_scene(gold["c2w"], gold["pts"], scale=True, rotate=True)
    np.testing.assert_allclose(np.asarray(c2w), gold["poses_ground_lookat"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(np.asarray(pts), gold["pts_ground_lookat"], rtol=0, atol=1e-6)
    c0, p0 = normalize_scene(gold["c2w"], gold["pts"], scale=False)
    assert np.array_equal(c0, gold["c2w"]) and np.array_equal(p0, gold["pts"])
