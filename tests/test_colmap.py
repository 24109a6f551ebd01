"""COLMAP binary readers (dogs_amd/colmap.py over dg_colmap_* in libdogs_hip.so; host code, no GPU) against what the
reference's own SceneManager (conerf/pycolmap/pycolmap/scene_manager.py:137-310) returned for the same files:
tests/golden/colmap/*.bin and tests/golden/colmap_expected.npz, made by tests/golden/make_colmap_golden.py.
Bit-exact on every field: camera intrinsics by model, image poses (R() from the quaternion), names (one empty),
points2D with the -1 (no 3D point) entries dropped, 3D points filtered at min_track_length = 3 with their tracks.
Plus the error behaviour on truncated / missing files."""
import os
import shutil

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden", "colmap")


@pytest.fixture(scope="module")
def scene():
    from dogs_amd.colmap import SceneManager
    m = SceneManager(GOLD, load_points=True)
    m.load()
    return m


@pytest.fixture(scope="module")
def exp():
    return dict(np.load(os.path.join(HERE, "golden", "colmap_expected.npz")))


def test_cameras(scene, exp):
    assert list(scene.cameras.keys()) == exp["camera_ids"].tolist()
    got = np.array([[c.fx, c.fy, c.cx, c.cy] for c in scene.cameras.values()])
    np.testing.assert_array_equal(got, exp["camera_fxfycxcy"])
    np.testing.assert_array_equal([[c.width, c.height] for c in scene.cameras.values()], exp["camera_wh"])
    np.testing.assert_array_equal([c.camera_type for c in scene.cameras.values()], exp["camera_types"])
    assert scene.cameras[9].k1 == 0.1 and scene.cameras[9].p2 == 0.002


def test_images(scene, exp):
    assert list(scene.images.keys()) == exp["image_ids"].tolist()
    assert [im.name for im in scene.images.values()] == exp["image_names"].tolist()
    assert "" in scene.name_to_image_id
    assert all(scene.name_to_image_id[im.name] == i for i, im in scene.images.items())
    np.testing.assert_array_equal([im.camera_id for im in scene.images.values()], exp["image_camera_ids"])
    np.testing.assert_array_equal(np.stack([im.R() for im in scene.images.values()]), exp["image_R"])
    np.testing.assert_array_equal(np.stack([im.tvec for im in scene.images.values()]), exp["image_tvec"])
    np.testing.assert_array_equal([len(im.point3D_ids) for im in scene.images.values()], exp["image_n2d"])
    np.testing.assert_array_equal(np.concatenate([im.points2D for im in scene.images.values()]),
                                  exp["image_points2D"])
    ids = np.concatenate([im.point3D_ids for im in scene.images.values()])
    np.testing.assert_array_equal(ids, exp["image_point3D_ids"])
    assert (ids != -1).all()


def test_points3d(scene, exp):
    np.testing.assert_array_equal(scene.points3D, exp["points3D"])
    np.testing.assert_array_equal(scene.point3D_ids.astype(np.int64), exp["point3D_ids"])
    np.testing.assert_array_equal(scene.point3D_colors.astype(np.int64), exp["point3D_colors"])
    np.testing.assert_array_equal(scene.point3D_errors, exp["point3D_errors"])
    tl = [len(scene.point3D_id_to_images[int(i)]) for i in scene.point3D_ids]
    np.testing.assert_array_equal(tl, exp["track_lengths"])
    assert min(tl) >= 3
    tr = np.concatenate([scene.point3D_id_to_images[int(i)] for i in scene.point3D_ids]).astype(np.int64)
    np.testing.assert_array_equal(tr, exp["tracks"])
    for i, pid in enumerate(scene.point3D_ids[:20]):
        assert scene.point3D_id_to_point3D_idx[int(pid)] == i and scene.point3D_idx_to_point3D_id[i] == int(pid)


def test_min_track_length_filter():
    from dogs_amd.colmap import read_points3D_binary
    all_ = read_points3D_binary(os.path.join(GOLD, "points3D.bin"), 0)
    assert len(all_["ids"]) == 300
    lens = np.diff(all_["track_offsets"].astype(np.int64))
    for k in range(0, 8):
        d = read_points3D_binary(os.path.join(GOLD, "points3D.bin"), k)
        keep = lens >= k
        np.testing.assert_array_equal(d["ids"], all_["ids"][keep])
        np.testing.assert_array_equal(d["xyz"], all_["xyz"][keep])


def test_errors(tmp_path):
    from dogs_amd.colmap import SceneManager, read_images_binary, read_points3D_binary
    with pytest.raises(IOError):
        SceneManager(str(tmp_path)).load()
    for name, reader in (("images.bin", read_images_binary), ("points3D.bin", read_points3D_binary)):
        raw = open(os.path.join(GOLD, name), "rb").read()
        for cut in (3, 40, len(raw) - 5):
            p = tmp_path / name
            p.write_bytes(raw[:cut])
            with pytest.raises(IOError):
                reader(str(p))
    # hostile lengths: a count whose byte size wraps around 2^64 must fail cleanly, not read past the mapping
    raw = bytearray(open(os.path.join(GOLD, "images.bin"), "rb").read())
    z = raw.index(0, 72)                                      # end of the first image's name
    for huge in (2 ** 62, 2 ** 64 // 24 + 1, 2 ** 64 - 1):
        raw[z + 1:z + 9] = np.array([huge], np.uint64).tobytes()
        (tmp_path / "images.bin").write_bytes(bytes(raw))
        with pytest.raises(IOError):
            read_images_binary(str(tmp_path / "images.bin"))
    raw = bytearray(open(os.path.join(GOLD, "points3D.bin"), "rb").read())
    for huge in (2 ** 61, 2 ** 64 // 8 + 1, 2 ** 64 - 1):
        raw[8 + 43:8 + 51] = np.array([huge], np.uint64).tobytes()
        (tmp_path / "points3D.bin").write_bytes(bytes(raw))
        with pytest.raises(IOError):
            read_points3D_binary(str(tmp_path / "points3D.bin"))
    bad = tmp_path / "cameras.bin"
    bad.write_bytes(np.array([1], np.uint64).tobytes() + np.array([1, 6], np.int32).tobytes() + b"\0" * 16)
    from dogs_amd.colmap import read_cameras_binary
    with pytest.raises(ValueError):
        read_cameras_binary(str(bad))
    shutil.rmtree(tmp_path, ignore_errors=True)


def test_colmap_views_and_block_export(tmp_path, exp):
    """load_colmap.py:226-273 view extraction on the golden model, then a block export (dataset_base.py:111-150)
    written and read back in the reference's format."""
    import torch
    from dogs_amd.blockio import MiniDataset, colmap_views, export_blocks
    v = colmap_views(GOLD, factor=2, scale=False)
    order = np.argsort(exp["image_names"])
    assert v["image_names"] == [exp["image_names"][i] for i in order]
    w2c = np.linalg.inv(v["camtoworlds"])
    np.testing.assert_allclose(w2c[:, :3, :3], exp["image_R"][order], rtol=0, atol=1e-12)
    np.testing.assert_allclose(w2c[:, :3, 3], exp["image_tvec"][order], rtol=0, atol=1e-12)
    cam_of = dict(zip(exp["camera_ids"].tolist(), exp["camera_fxfycxcy"]))
    for i, j in enumerate(order):
        fx, fy, cx, cy = cam_of[int(exp["image_camera_ids"][j])]
        np.testing.assert_array_equal(v["intrinsics"][i], [[fx / 2, 0, cx / 2], [0, fy / 2, cy / 2], [0, 0, 1]])
        assert v["image_index_to_image_id"][i] == int(exp["image_ids"][j])
    np.testing.assert_array_equal(v["points3d"], exp["points3D"])
    # with load_colmap's defaults the scene is normalised (dogs_amd.normalize, pinned in tests/test_normalize.py)
    from dogs_amd.normalize import normalize_scene
    vn = colmap_views(GOLD, factor=2)
    c_ref, p_ref = normalize_scene(v["camtoworlds"], v["points3d"])
    np.testing.assert_allclose(vn["camtoworlds"], np.asarray(c_ref, dtype=np.float64), rtol=0, atol=0)
    np.testing.assert_allclose(vn["points3d"], np.asarray(p_ref, dtype=np.float64), rtol=0, atol=0)
    blocks = {0: [np.array([0, 1, 2, 3])], 1: [np.array([2, 3, 4, 5])]}   # overlapping blocks, image 3 is validation
    out = export_blocks(str(tmp_path), v, blocks, val_indices=[3])
    assert [len(d) for d in out] == [3, 3]
    for b, d in enumerate(out):
        back = MiniDataset().read(str(tmp_path / f"block_{b}"), block_id=b)
        assert len(back) == len(d) and back.current_block == b
        torch.testing.assert_close(back.camtoworlds, d.camtoworlds)
        for c0, c1 in zip(d.cameras, back.cameras):
            assert c0.state_dict().keys() == c1.state_dict().keys()
            torch.testing.assert_close(c1.world_to_camera, c0.world_to_camera)
            assert (c1.image_index, c1.width, c1.fx, c1.image_path) == (c0.image_index, c0.width, c0.fx,
                                                                          c0.image_path)
            rc = c1.raster_camera()
            assert rc.width == c1.width and torch.isfinite(rc.projective_matrix).all()
    # image_index is the position in the block (compose_cameras); the image paths name the global images 2, 4, 5
    assert [c.image_index for c in out[1].cameras] == [0, 1, 2]
    assert [c.image_path for c in out[1].cameras] == [v["image_names"][i] for i in (2, 4, 5)]
    np.testing.assert_allclose(out[0].cameras[1].world_to_camera.numpy(), w2c[1].astype(np.float32), atol=1e-5)
