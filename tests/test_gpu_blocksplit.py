"""Grid2D block split on the GPU (dg_points_in_boxes2d, dogs_amd/blocksplit.py) against the CPU restatement
(oracle/blocksplit_oracle.py; reference cluster.py:73-199, utils.py:64-206, load_colmap.py:98-177).
Bit-exact: membership lists, labels, counts, transformed coordinates, cells, expanded cells and the OBB transform.
Parity with the reference itself is unpinned (trimesh absent, no reference fixture)."""
import math
import os

import numpy as np
import pytest
import torch

from oracle import blocksplit_oracle as O

pytestmark = pytest.mark.gpu


def _cloud(n, seed, w=8.0, h=3.0, theta=0.7):
    rng = np.random.default_rng(seed)
    u = rng.normal(size=(n, 2)) * [w / 4, h / 4]
    c, s = math.cos(theta), math.sin(theta)
    xy = u @ np.array([[c, -s], [s, c]]).T + [120.0, -40.0]
    z = rng.normal(size=(n, 1))
    return np.concatenate([xy, z], axis=1)


def test_points_in_boxes_matches_oracle(hip_device):
    from dogs_amd import blocksplit as G
    p = _cloud(300_001, 0)
    T, _ = O.oriented_bounds_2D(p[:2000, :2])
    q = O.transform_points(p[:, :2], T)
    rng = np.random.default_rng(1)
    boxes = []
    for _ in range(37):
        a = rng.uniform(q.min(0), q.max(0))
        b = a + rng.uniform(0.1, 3.0, size=2)
        boxes.append(np.array([[a[0], a[1]], [b[0], b[1]]]))
    boxes.append(np.array([[q[5, 0], q[5, 1]], [q[5, 0], q[5, 1]]]))      # a point exactly on a degenerate box
    r = G.points_in_boxes2d(p, boxes, T, labels=True, transformed=True, device=hip_device)
    np.testing.assert_array_equal(r["transformed"].cpu().numpy(), q)
    lab = np.zeros(len(p), np.uint8)
    for k, b in enumerate(boxes):
        ref = O.points_in_bbox2D(p, b, T)
        np.testing.assert_array_equal(r["members"][k].cpu().numpy(), ref)
        assert r["counts"][k] == len(ref)
        lab[ref] = k
    assert 5 in r["members"][-1].cpu().numpy()
    np.testing.assert_array_equal(r["labels"].cpu().numpy(), lab)


def test_points_in_boxes_edges(hip_device):
    from dogs_amd import blocksplit as G
    r = G.points_in_boxes2d(np.zeros((0, 3)), [np.array([[0, 0], [1, 1]])], device=hip_device)
    assert r["counts"].tolist() == [0] and r["members"][0].numel() == 0
    grid = np.stack(np.meshgrid(np.arange(8.0), np.arange(8.0)), -1).reshape(-1, 2)
    boxes = [np.array([[x, y], [x, y]]) for y in range(8) for x in range(8)]  # 64 boxes, one point each
    r = G.points_in_boxes2d(grid, boxes, labels=True, device=hip_device)
    assert [m.tolist() for m in r["members"]] == [[i] for i in range(64)]
    np.testing.assert_array_equal(r["labels"].cpu().numpy(), np.arange(64))
    with pytest.raises(RuntimeError):
        G.points_in_boxes2d(grid, boxes + boxes[:1], device=hip_device)
    nan = np.array([[np.nan, 0.0], [0.5, 0.5]])
    assert G.points_in_bbox2D(nan, np.array([[0, 0], [1, 1]])).tolist() == [1]


@pytest.mark.parametrize("mx,my,prior", [(2, 2, False), (3, 1, False), (2, 2, True), (4, 3, False)])
def test_grid2d_clustering_matches_oracle(hip_device, mx, my, prior):
    from dogs_amd import blocksplit as G
    p = _cloud(50_000, 2 + mx)
    lab_o, cells_o, exp_o, T_o = O.Grid2DClustering(p, mx=mx, my=my, use_prior_center=prior)
    lab, cells, exp, T = G.Grid2DClustering(p, mx=mx, my=my, use_prior_center=prior)
    np.testing.assert_array_equal(T, T_o)
    for a, b in zip(cells, cells_o):
        np.testing.assert_array_equal(a, b)
    for a, b in zip(exp, exp_o):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(lab, lab_o)


def test_cluster_points_and_images(hip_device, tmp_path):
    from dogs_amd import blocksplit as G
    pts = _cloud(40_000, 9)
    cols = np.random.default_rng(3).integers(0, 256, size=(len(pts), 3)).astype(np.uint8)
    bb, eb, T = G.cluster_points_in_grid(pts, cols, str(tmp_path), [1.2, 1.2], mx=2, my=2)
    _, cells_o, exp_o, T_o = O.Grid2DClustering(pts, scale_factor=[1.2, 1.2], p0=0.00001, p1=0.99999, mx=2, my=2)
    np.testing.assert_array_equal(T, T_o)
    np.testing.assert_array_equal(eb, np.stack(exp_o))
    for k in range(4):
        sel = O.points_in_bbox2D(pts, exp_o[k], T_o)
        blob = open(tmp_path / f"points3D_{k}.ply", "rb").read()
        head, body = blob.split(b"end_header\n", 1)
        assert f"element vertex {len(sel)}".encode() in head
        rec = np.frombuffer(body, dtype=[("xyz", "<f4", 3), ("n", "<f4", 3), ("rgb", "u1", 3)])
        np.testing.assert_array_equal(rec["xyz"], pts[sel].astype(np.float32))
        np.testing.assert_array_equal(rec["rgb"], cols[sel])
    # cameras: 200 poses over the same area
    c2w = np.tile(np.eye(4), (200, 1, 1))
    c2w[:, :3, 3] = _cloud(200, 11)
    ids = {i: 1000 + i for i in range(200)}
    blocks, bb, eb, T = G.cluster_image_in_grid(c2w, str(tmp_path), np.arange(200) * 2, [1.1, 1.1], ids, 1, 2, 2)
    lab_o, _, exp_o, T_o = O.Grid2DClustering(c2w[:, :3, 3], scale_factor=[1.1, 1.1], p0=0, p1=1, mx=2, my=2)
    lines = open(tmp_path / "cluster.txt").read().split("\n")
    assert lines[:200] == [f"{1000 + i} {lab_o[i]}" for i in range(200)]
    for k in range(4):
        np.testing.assert_array_equal(blocks[k][0], 2 * O.points_in_bbox2D(c2w[:, :3, 3], exp_o[k], T_o))


def test_colmap_to_block_folders(hip_device, tmp_path):
    """The whole block-preprocessing path on the golden COLMAP model: native binary readers -> sorted views
    (load_colmap.py:226-273) -> Grid2D split of cameras and points on the GPU (:412-425) -> per-block folders in
    MiniDataset's format (:459-487, dataset_base.py:111-124), read back."""
    import os
    from dogs_amd import blocksplit
    from dogs_amd.blockio import MiniDataset, colmap_views, export_blocks
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "colmap")
    v = colmap_views(gold, scale=False)
    n = len(v["image_names"])
    bids, cb, ecb, T = blocksplit.cluster_image_in_grid(v["camtoworlds"], str(tmp_path), np.arange(n),
                                                        [1.0, 1.0, 1.0], v["image_index_to_image_id"], 2, 2, 1)
    pb, epb, _ = blocksplit.cluster_points_in_grid(v["points3d"], v["colors"], str(tmp_path), [1.0, 1.0, 1.0], 2, 2, 1,
                                                   False, T)
    assert len(bids) == 2 and os.path.exists(tmp_path / "cluster.txt") and os.path.exists(tmp_path / "points3D_0.ply")
    # the image sets are the oracle's (strict box test: a camera on an expanded cell's edge belongs to no block)
    c = v["camtoworlds"][:, :3, -1]
    _, _, exp_cells, To = O.Grid2DClustering(c, scale_factor=(1.0, 1.0), p0=0, p1=1, mx=2, my=1, num_blocks=2)
    for k, e in enumerate(exp_cells):
        assert np.concatenate(bids[k]).tolist() == list(O.points_in_bbox2D(c[:, :2], e, To))
    out = export_blocks(str(tmp_path / "blocks"), v, bids)
    for b, d in enumerate(out):
        back = MiniDataset().read(str(tmp_path / "blocks" / f"block_{b}"), block_id=b)
        assert [c.image_path for c in back.cameras] == [v["image_names"][i] for i in sorted(np.concatenate(bids[b]))]
        assert [c.image_index for c in back.cameras] == list(range(len(back.cameras)))
