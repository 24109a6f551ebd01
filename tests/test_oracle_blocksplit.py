"""Known answers of the Grid2D block-split restatement (oracle/blocksplit_oracle.py; reference cluster.py:73-199,
utils.py:64-206).  trimesh is absent and the reference holds no fixture for the split: these cases pin the
restatement (parity with the reference itself unpinned)."""
import math

import numpy as np
import pytest

from oracle import blocksplit_oracle as B


def _rotated_rect(w, h, theta, n=4000, seed=0, centre=(3.0, -2.0)):
    rng = np.random.default_rng(seed)
    u = rng.uniform(-0.5, 0.5, size=(n, 2)) * [w, h]
    c, s = math.cos(theta), math.sin(theta)
    R = np.array([[c, -s], [s, c]])
    return u @ R.T + np.asarray(centre)


def test_points_in_bbox2D_is_closed_and_ascending():
    p = np.array([[0.0, 0.0], [1.0, 1.0], [1.0000001, 0.5], [0.5, 0.5], [-1e-300, 0.0]])
    idx = B.points_in_bbox2D(p, np.array([[0.0, 0.0], [1.0, 1.0]]))
    assert idx.tolist() == [0, 1, 3]
    assert idx.dtype == np.int64


def test_points_in_bbox2D_in_obb_frame():
    T = np.array([[0.0, 1.0, 0.0], [-1.0, 0.0, 0.0], [0, 0, 1]])        # (x, y) -> (y, -x)
    p = np.array([[0.5, 2.0], [2.0, 0.5]])
    assert B.points_in_bbox2D(p, np.array([[1.5, -1.0], [2.5, 0.0]]), T).tolist() == [0]


def test_oriented_bounds_recovers_a_rotated_rectangle():
    for theta in (0.3, -1.1, 2.0):
        p = _rotated_rect(4.0, 1.0, theta, seed=1)
        T, ext = B.oriented_bounds_2D(p)
        assert ext[0] >= ext[1]                               # long side on x
        np.testing.assert_allclose(ext, [4.0, 1.0], atol=0.02)
        q = B.transform_points(p, T)
        np.testing.assert_allclose(q.min(0), -ext / 2, atol=1e-9)
        np.testing.assert_allclose(q.max(0), ext / 2, atol=1e-9)


def test_compute_bounding_box2D_extremes_and_expand():
    p = np.array([[0.0, 0.0], [2.0, 2.0], [1.0, 0.5]])
    box = B.compute_bounding_box2D(p, [1.0, 1.0], -1.0, 1.0, 0, 1)
    np.testing.assert_allclose(box, [[0, 0, -1], [2, 2, 1]], atol=1e-12)
    e = B.expand_bounding_box([0.0, 0.0, 2.0, 2.0], [1.2, 1.2])
    s = float(np.float32(1.2))                                # torch.tensor([1.2]) is float32
    np.testing.assert_allclose(e, [[1 - s, 1 - s], [1 + s, 1 + s]], rtol=0, atol=1e-15)


def test_grid2d_split_labels_and_cells():
    p = _rotated_rect(8.0, 4.0, 0.4, n=20000, seed=2)
    labels, cells, exp_cells, T = B.Grid2DClustering(p, mx=2, my=2, p0=0, p1=1)
    assert len(cells) == 4 and len(exp_cells) == 4
    counts = np.bincount(labels, minlength=4)
    assert counts.sum() == len(p)
    assert np.all(np.abs(counts - len(p) / 4) < 0.05 * len(p))   # uniform cloud: four nearly equal blocks
    for c, e in zip(cells, exp_cells):
        assert np.all(e[0, :2] < c[0, :2]) and np.all(e[1, :2] > c[1, :2])   # expanded outwards
    # the last cell containing a point wins (cells share their edges)
    for k in range(4):
        inside = B.points_in_bbox2D(p, cells[k], T)
        assert np.all(labels[inside] >= k)


def test_prior_center_cells():
    p = _rotated_rect(8.0, 4.0, 0.0, n=2000, seed=3, centre=(0.0, 0.0))
    cells, _ = B.Grid2DXY(p, mx=2, my=2, use_prior_center=True)
    assert len(cells) == 4
    assert cells[0][1, 0] == 0.0 and cells[3][0, 1] == 0.0


def test_empty_division_raises():
    p = np.array([[0.0, 0.0], [0.0, 1.0], [10.0, 0.0], [10.0, 1.0], [0.0, 0.5], [10.0, 0.5]])
    with pytest.raises(IndexError):
        B.Grid2DXY(p, mx=3, my=1, p0=0, p1=1, transform_world_to_obb=np.eye(3))
