"""COLMAP binary model loading for the block split, over the native readers of
libdogs_hip.so (dg_colmap_*; host code).

`SceneManager` mirrors the parts of conerf/pycolmap/pycolmap/scene_manager.py that load_colmap (load_colmap.py:
221-226) uses -- `load()`, `cameras`, `images`, `name_to_image_id`, `points3D`, `point3D_ids`, `point3D_colors`,
`point3D_errors`, `point3D_id_to_point3D_idx`, `point3D_idx_to_point3D_id`, `point3D_id_to_images` -- with the
reference's types (float64 arrays, OrderedDicts keyed by COLMAP ids, cameras with fx/fy/cx/cy, images with q, tvec,
R()).  The reference parses each record with Python struct calls; here each file is one mapped two-pass C++ walk,
and the per-record Python objects are built from whole arrays.  Text models (cameras.txt ...) are not handled.
"""
from __future__ import annotations

import ctypes as C
import os
from collections import OrderedDict
from collections.abc import Mapping

import numpy as np

from . import _lib

CAMERA_MODELS = {0: "SIMPLE_PINHOLE", 1: "PINHOLE", 2: "SIMPLE_RADIAL", 3: "RADIAL", 4: "OPENCV"}
NUM_PARAMS = {0: 3, 1: 4, 2: 4, 3: 5, 4: 8}


def _check(rc: int, path: str) -> None:
    if rc == 1:
        raise IOError(f"cannot open {path}")
    if rc == 2:
        raise IOError(f"{path}: truncated or malformed COLMAP binary file")
    if rc == 3:
        raise ValueError(f"{path}: camera type not supported")
    if rc:
        raise RuntimeError(f"{path}: COLMAP reader failed ({rc})")


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class Camera:
    """pycolmap Camera (camera.py): parameters by model."""

    def __init__(self, type_: int, width: int, height: int, params):
        self.width, self.height = int(width), int(height)
        self.camera_type = int(type_)
        p = [float(x) for x in params]
        if type_ == 0:
            self.fx, self.cx, self.cy = p
            self.fy = self.fx
        elif type_ == 1:
            self.fx, self.fy, self.cx, self.cy = p
        elif type_ == 2:
            self.fx, self.cx, self.cy, self.k1 = p
            self.fy = self.fx
        elif type_ == 3:
            self.fx, self.cx, self.cy, self.k1, self.k2 = p
            self.fy = self.fx
        elif type_ == 4:
            self.fx, self.fy, self.cx, self.cy = p[:4]
            self.k1, self.k2, self.p1, self.p2 = p[4:]
        else:
            raise ValueError("Camera type not supported")

    @staticmethod
    def GetNumParams(type_):  # noqa: N802 - the reference's name
        return NUM_PARAMS[type_]


class Quaternion:
    def __init__(self, q):
        self.q = np.asarray(q, dtype=np.float64).copy()

    def ToR(self):  # noqa: N802 - rotation.py:180-190
        q = self.q
        return np.eye(3) + 2 * np.array((
            (-q[2] * q[2] - q[3] * q[3], q[1] * q[2] - q[3] * q[0], q[1] * q[3] + q[2] * q[0]),
            (q[1] * q[2] + q[3] * q[0], -q[1] * q[1] - q[3] * q[3], q[2] * q[3] - q[1] * q[0]),
            (q[1] * q[3] - q[2] * q[0], q[2] * q[3] + q[1] * q[0], -q[1] * q[1] - q[2] * q[2])))


class Image:
    """pycolmap Image (image.py)."""

    def __init__(self, name, camera_id, q, tvec):
        self.name, self.camera_id, self.q, self.tvec = name, camera_id, q, tvec
        self.points2D = np.empty((0, 2), dtype=np.float64)
        self.point3D_ids = np.empty((0,), dtype=np.uint64)

    def R(self):  # noqa: N802
        return self.q.ToR()

    def C(self):  # noqa: N802
        return -self.R().T.dot(self.tvec)

    @property
    def t(self):
        return self.tvec


def read_cameras_binary(path: str) -> dict:
    """{'ids', 'models', 'wh', 'params'} arrays of cameras.bin (params zero-padded to 8)."""
    L = _lib.load()
    n = C.c_uint64(0)
    _check(L.dg_colmap_cameras(path.encode(), C.byref(n), None, None, None, None), path)
    k = int(n.value)
    out = {"ids": np.zeros(k, np.uint32), "models": np.zeros(k, np.int32), "wh": np.zeros((k, 2), np.uint64),
           "params": np.zeros((k, 8), np.float64)}
    _check(L.dg_colmap_cameras(path.encode(), C.byref(n), _ptr(out["ids"]), _ptr(out["models"]), _ptr(out["wh"]),
                               _ptr(out["params"])), path)
    return out


def read_images_binary(path: str) -> dict:
    """{'ids', 'qvec', 'tvec', 'camera_ids', 'names', 'p2d_offsets', 'xy', 'point3D_ids'} of images.bin."""
    L = _lib.load()
    n, nb, m = C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
    args = [None] * 8
    _check(L.dg_colmap_images(path.encode(), C.byref(n), C.byref(nb), C.byref(m), *args), path)
    k, nbytes, np2 = int(n.value), int(nb.value), int(m.value)
    ids, qt = np.zeros(k, np.uint32), np.zeros((k, 7), np.float64)
    cams, noff = np.zeros(k, np.uint32), np.zeros(k + 1, np.uint64)
    names = np.zeros(max(nbytes, 1), np.uint8)
    poff, xy, pid = np.zeros(k + 1, np.uint64), np.zeros((max(np2, 1), 2), np.float64), np.zeros(max(np2, 1), np.int64)
    _check(L.dg_colmap_images(path.encode(), C.byref(n), C.byref(nb), C.byref(m), _ptr(ids), _ptr(qt), _ptr(cams),
                              _ptr(noff), _ptr(names), _ptr(poff), _ptr(xy), _ptr(pid)), path)
    raw = names.tobytes()
    return {"ids": ids, "qvec": qt[:, :4], "tvec": qt[:, 4:], "camera_ids": cams,
            "names": [raw[int(noff[i]):int(noff[i + 1])].decode() for i in range(k)],
            "p2d_offsets": poff, "xy": xy[:np2], "point3D_ids": pid[:np2]}


def read_points3D_binary(path: str, min_track_length: int = 3) -> dict:  # noqa: N802 - COLMAP's name
    """{'ids', 'xyz', 'rgb', 'errors', 'track_offsets', 'tracks'} of the points with track_len >= min_track_length."""
    L = _lib.load()
    n, t = C.c_uint64(0), C.c_uint64(0)
    _check(L.dg_colmap_points3d(path.encode(), int(min_track_length), C.byref(n), C.byref(t), *([None] * 6)), path)
    k, nt = int(n.value), int(t.value)
    out = {"ids": np.zeros(k, np.uint64), "xyz": np.zeros((k, 3), np.float64), "rgb": np.zeros((k, 3), np.uint8),
           "errors": np.zeros(k, np.float64), "track_offsets": np.zeros(k + 1, np.uint64),
           "tracks": np.zeros((max(nt, 1), 2), np.uint32)}
    _check(L.dg_colmap_points3d(path.encode(), int(min_track_length), C.byref(n), C.byref(t), _ptr(out["ids"]),
                                _ptr(out["xyz"]), _ptr(out["rgb"]), _ptr(out["errors"]), _ptr(out["track_offsets"]),
                                _ptr(out["tracks"])), path)
    out["tracks"] = out["tracks"][:nt]
    return out


class _TrackMap(Mapping):
    """point3D_id -> [track_len, 2] (image_id, point2D_idx) view of the flat track array: the reference's dict of
    per-point arrays, sliced on access instead of built per point."""

    def __init__(self, idx_of: dict, offsets: np.ndarray, tracks: np.ndarray):
        self._idx, self._off, self._tr = idx_of, offsets, tracks

    def __getitem__(self, pid):
        i = self._idx[int(pid)]
        return self._tr[self._off[i]:self._off[i + 1]]

    def __iter__(self):
        return iter(self._idx)

    def __len__(self):
        return len(self._idx)


class SceneManager:
    """The loading part of pycolmap's SceneManager over the native readers (binary models)."""

    def __init__(self, colmap_results_folder: str, image_path: str | None = None, load_points: bool = False):
        self.folder = colmap_results_folder
        if not self.folder.endswith("/"):
            self.folder += "/"
        self.image_path = image_path
        self.load_points = load_points
        self.cameras = OrderedDict()
        self.images = OrderedDict()
        self.name_to_image_id = {}
        self.last_camera_id = 0
        self.last_image_id = 0
        self.points3D = np.zeros((0, 3))
        self.point3D_ids = np.zeros(0, np.uint64)
        self.point3D_colors = np.zeros((0, 3), np.uint8)
        self.point3D_errors = np.zeros(0)
        self.point3D_id_to_point3D_idx = {}
        self.point3D_idx_to_point3D_id = {}
        self.point3D_id_to_images = {}

    def load(self):
        self.load_cameras()
        self.load_images()
        if self.load_points:
            self.load_points3D()

    def _path(self, name: str, input_file: str | None) -> str:
        p = input_file or self.folder + name
        if not os.path.exists(p):
            raise IOError(f"no {name} found in {self.folder} (binary models only)")
        return p

    def load_cameras(self, input_file: str | None = None):
        c = read_cameras_binary(self._path("cameras.bin", input_file))
        self.cameras = OrderedDict()
        for i in range(len(c["ids"])):
            m = int(c["models"][i])
            cid = int(c["ids"][i])
            self.cameras[cid] = Camera(m, int(c["wh"][i, 0]), int(c["wh"][i, 1]), c["params"][i, :NUM_PARAMS[m]])
            self.last_camera_id = max(self.last_camera_id, cid)

    def load_images(self, input_file: str | None = None):
        d = read_images_binary(self._path("images.bin", input_file))
        self.images = OrderedDict()
        off = d["p2d_offsets"].astype(np.int64)
        for i in range(len(d["ids"])):
            iid = int(d["ids"][i])
            im = Image(d["names"][i], int(d["camera_ids"][i]), Quaternion(d["qvec"][i]), d["tvec"][i].copy())
            im.points2D = d["xy"][off[i]:off[i + 1]].copy()
            im.point3D_ids = d["point3D_ids"][off[i]:off[i + 1]].copy()
            self.images[iid] = im
            self.name_to_image_id[im.name] = iid
            self.last_image_id = max(self.last_image_id, iid)

    def load_points3D(self, input_file: str | None = None, min_track_length: int = 3):  # noqa: N802
        d = read_points3D_binary(self._path("points3D.bin", input_file), min_track_length)
        self.points3D = d["xyz"]
        self.point3D_ids = d["ids"]
        self.point3D_colors = d["rgb"]
        self.point3D_errors = d["errors"]
        ids = d["ids"].tolist()
        self.point3D_id_to_point3D_idx = dict(zip(ids, range(len(ids))))
        self.point3D_idx_to_point3D_id = dict(enumerate(ids))
        self.point3D_id_to_images = _TrackMap(self.point3D_id_to_point3D_idx, d["track_offsets"].astype(np.int64),
                                              d["tracks"])
