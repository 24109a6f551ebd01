"""Times the native COLMAP points3D.bin reader (dogs_amd/colmap.py) against the reference's SceneManager (imported
from /root/reference when present, this container only) on a synthetic city-scale file.

usage: python tools/colmap_bench.py [n_points] [track_len]"""
import os
import sys
import tempfile
import time

import numpy as np


def write_points(path, n, tl, seed=0):
    rng = np.random.default_rng(seed)
    rec = np.dtype([("id", "<u8"), ("xyz", "<f8", 3), ("rgb", "u1", 3), ("err", "<f8"), ("tl", "<u8"),
                    ("track", "<u4", 2 * tl)])
    a = np.zeros(n, rec)
    a["id"] = np.arange(n) * 3 + 1
    a["xyz"] = rng.standard_normal((n, 3))
    a["rgb"] = rng.integers(0, 256, (n, 3))
    a["err"] = rng.random(n)
    a["tl"] = tl
    a["track"] = rng.integers(0, 5000, (n, 2 * tl))
    with open(path, "wb") as f:
        f.write(np.uint64(n).tobytes())
        f.write(a.tobytes())


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    tl = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from dogs_amd.colmap import SceneManager, read_points3D_binary
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "points3D.bin")
        write_points(p, n, tl)
        t = time.perf_counter()
        r = read_points3D_binary(p)
        t_arr = time.perf_counter() - t
        m = SceneManager(d)
        t = time.perf_counter()
        m.load_points3D()
        t_nat = time.perf_counter() - t
        line = {"n_points": n, "track_len": tl, "MB": os.path.getsize(p) / 1e6, "native_arrays_s": round(t_arr, 4),
                "native_scenemanager_s": round(t_nat, 3)}
        if os.path.isdir("/root/reference"):
            sys.path.insert(0, "/root/reference")
            from conerf.pycolmap.pycolmap.scene_manager import SceneManager as RefSM
            rm = RefSM(d + "/")
            t = time.perf_counter()
            rm.load_points3D()
            line["reference_s"] = round(time.perf_counter() - t, 3)
            assert np.array_equal(rm.points3D, r["xyz"]) and np.array_equal(rm.point3D_errors, r["errors"])
        print(line)


if __name__ == "__main__":
    main()
