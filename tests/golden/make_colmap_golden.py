"""Writes a small synthetic COLMAP binary model (cameras.bin, images.bin, points3D.bin) in the layout
SceneManager reads (conerf/pycolmap/pycolmap/scene_manager.py:137-310 / _save_*_bin), loads it with the REFERENCE's
own SceneManager (imported from /root/reference by path, in this container only), and freezes what it returns into
tests/golden/colmap_expected.npz -- the fixture the native readers (dogs_amd/colmap.py) are checked against.
Edge cases: every camera model, image names of several lengths (one empty), points2D without a 3D point (-1),
points with track lengths 0..6 around the min_track_length = 3 filter.

usage: python tests/golden/make_colmap_golden.py   (run from the repo root, where /root/reference exists)"""
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "colmap")


def write_model(out):
    rng = np.random.default_rng(7)
    os.makedirs(out, exist_ok=True)
    cams = [(1, 0, 640, 480, [500.0, 320.0, 240.0]), (3, 1, 1920, 1080, [1600.0, 1610.5, 960.25, 540.75]),
            (4, 2, 800, 600, [700.0, 400.0, 300.0, 0.01]), (7, 3, 1024, 768, [900.0, 512.0, 384.0, 0.02, -0.003]),
            (9, 4, 3840, 2160, [3000.0, 3001.0, 1920.0, 1080.0, 0.1, -0.02, 0.001, 0.002])]
    with open(os.path.join(out, "cameras.bin"), "wb") as f:
        f.write(struct.pack("<Q", len(cams)))
        for cid, model, w, h, params in cams:
            f.write(struct.pack("<IiQQ", cid, model, w, h))
            f.write(struct.pack(f"<{len(params)}d", *params))
    names = ["a.jpg", "dir/img_0002.png", "", "long_name_" + "x" * 40 + ".jpg", "e.JPG", "f.jpg"]
    with open(os.path.join(out, "images.bin"), "wb") as f:
        f.write(struct.pack("<Q", len(names)))
        for i, nm in enumerate(names):
            q = rng.standard_normal(4)
            q /= np.linalg.norm(q)
            t = rng.standard_normal(3) * 5
            f.write(struct.pack("<I4d3dI", 10 + 3 * i, *q, *t, cams[i % len(cams)][0]))
            f.write(nm.encode() + b"\x00")
            n2 = int(rng.integers(0, 12))
            f.write(struct.pack("<Q", n2))
            for _ in range(n2):
                pid = -1 if rng.random() < 0.3 else int(rng.integers(0, 2 ** 40))
                f.write(struct.pack("<ddq", *(rng.random(2) * 1000), pid))
    with open(os.path.join(out, "points3D.bin"), "wb") as f:
        n = 300
        f.write(struct.pack("<Q", n))
        for i in range(n):
            tl = int(rng.integers(0, 7))
            f.write(struct.pack("<Q3d3BdQ", 1000 + 7 * i, *(rng.standard_normal(3) * 10),
                                *rng.integers(0, 256, 3), float(rng.random()), tl))
            f.write(np.asarray(rng.integers(0, 2 ** 31, 2 * tl), dtype=np.uint32).tobytes())


def main():
    write_model(OUT)
    sys.path.insert(0, "/root/reference")
    from conerf.pycolmap.pycolmap.scene_manager import SceneManager
    m = SceneManager(OUT + "/", load_points=True)
    m.load()
    exp = {}
    exp["camera_ids"] = np.array(list(m.cameras.keys()), np.int64)
    exp["camera_fxfycxcy"] = np.array([[c.fx, c.fy, c.cx, c.cy] for c in m.cameras.values()])
    exp["camera_wh"] = np.array([[c.width, c.height] for c in m.cameras.values()], np.int64)
    exp["camera_types"] = np.array([c.camera_type for c in m.cameras.values()], np.int64)
    exp["image_ids"] = np.array(list(m.images.keys()), np.int64)
    exp["image_names"] = np.array([im.name for im in m.images.values()])
    exp["image_camera_ids"] = np.array([im.camera_id for im in m.images.values()], np.int64)
    exp["image_R"] = np.stack([im.R() for im in m.images.values()])
    exp["image_tvec"] = np.stack([im.tvec for im in m.images.values()])
    exp["image_n2d"] = np.array([len(im.point3D_ids) for im in m.images.values()], np.int64)
    exp["image_points2D"] = np.concatenate([im.points2D.reshape(-1, 2) for im in m.images.values()])
    exp["image_point3D_ids"] = np.concatenate([np.asarray(im.point3D_ids, np.int64).reshape(-1)
                                               for im in m.images.values()])
    exp["points3D"] = m.points3D
    exp["point3D_ids"] = np.asarray(m.point3D_ids, np.int64)
    exp["point3D_colors"] = np.asarray(m.point3D_colors, np.int64)
    exp["point3D_errors"] = m.point3D_errors
    exp["track_lengths"] = np.array([len(m.point3D_id_to_images[int(i)]) for i in m.point3D_ids], np.int64)
    exp["tracks"] = np.concatenate([m.point3D_id_to_images[int(i)] for i in m.point3D_ids]).astype(np.int64)
    np.savez(os.path.join(HERE, "colmap_expected.npz"), **exp)
    print({k: v.shape for k, v in exp.items()})


if __name__ == "__main__":
    main()
