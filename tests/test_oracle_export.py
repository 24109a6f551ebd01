"""Known answers of the export restatement (oracle/export_oracle.py): the PLY header and record layout of
save_ply, the record layout and ordering of save_splat (gaussian_splat_model.py:616-708)."""
import numpy as np

from oracle import export_oracle as X


def test_ply_header_and_records():
    h = X.ply_header(2).decode()
    assert h.startswith("ply\nformat binary_little_endian 1.0\nelement vertex 2\nproperty float x\n")
    assert h.endswith("property uchar blue\nend_header\n")
    body = X.ply_body(np.array([[1, 2, 3], [4, 5, 6]], np.float32), np.array([[0, 0, 0], [10, -10, 0]], np.float32))
    assert len(body) == 2 * 27
    rec = np.frombuffer(body, dtype=X.FIELDS)
    np.testing.assert_array_equal(rec["x"], [1, 4])
    np.testing.assert_array_equal(rec["nz"], [0, 0])
    assert (rec["red"][0], rec["green"][0], rec["blue"][0]) == (127, 127, 127)   # 0.5 * 255
    assert rec["green"][1] == 0    # clamp_min(0)


def test_splat_order_and_layout():
    xyz = np.array([[0, 0, 0], [1, 1, 1]], np.float32)
    scaling = np.array([[-3, -3, -3], [-1, -1, -1]], np.float32)    # the larger Gaussian sorts first
    opacity = np.array([[0.0], [0.0]], np.float32)
    rot = np.array([[2, 0, 0, 0], [0, 0, 0, 1]], np.float32)
    dc = np.zeros((2, 1, 3), np.float32)
    p, s, c, q = X.splat_records(X.splat_body(xyz, scaling, opacity, rot, dc))
    np.testing.assert_array_equal(p, [[1, 1, 1], [0, 0, 0]])
    np.testing.assert_allclose(s[0], np.exp(np.float32(-1)), rtol=1e-6)
    np.testing.assert_array_equal(c[:, 3], [127, 127])          # sigmoid(0) * 255
    np.testing.assert_array_equal(q, [[128, 128, 128, 255], [255, 128, 128, 128]])


def test_bounding_box_and_fuse():
    rng = np.random.default_rng(0)
    pts = rng.uniform(-1, 1, (1000, 3))
    box = X.bounding_box2d(pts[:, :2], [1.0, 1.0], -1.0, 1.0, 0.0, 1.0)
    np.testing.assert_allclose(box[0, :2], pts[:, :2].min(0))
    np.testing.assert_allclose(box[1, :2], pts[:, :2].max(0))
    fused, boxes = X.fuse_blocks([{"xyz": pts}], [np.array([[0, 0, -1], [1, 1, 1]])], np.eye(3))
    assert len(boxes) == 1 and (fused["xyz"][:, :2] >= 0).all()
