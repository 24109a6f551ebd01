"""Block export around the Grid2D split: COLMAP model -> sorted views -> per-block view sets ->
the on-disk block folders the ADMM block trainers read.

* `colmap_views` restates load_colmap.py:226-313: load the binary model through the native readers
  (dogs_amd/colmap.py), build per image K = [[fx/f, 0, cx/f], [0, fy/f, cy/f], [0, 0, 1]] and w2c = [R | t; 0 0 0 1],
  invert to camera-to-world, sort by image name, map sorted index -> COLMAP image id, then (scale / rotate, the
  reference's defaults) the scene normalisation (dogs_amd.normalize: similarity_from_cameras + normalize_poses), so
  the Grid2D split runs in the reference's frame.  Image/normal file discovery is dataset plumbing, not restated.
* `block_views` restates the per-block selection of load_colmap.py:459-487 (block members in image order, validation
  indices removed, poses/intrinsics as float32 tensors).
* `MiniDataset` writes/reads the reference's block folder format (dataset_base.py:96-150): cameras/camera_{i}.pt, one
  state dict per camera as Camera.compose_state_dict (geometry/camera.py:165-185: world_to_camera 4x4, image_index,
  width, height, image_path, fx, fy, cx, cy), plus cameratoworlds.pt.  Reading uses torch.load(weights_only=True):
  the files hold tensors, numbers and strings only.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np
import torch

from .camera import RasterCamera, make_camera
from .colmap import SceneManager


def colmap_views(colmap_dir: str, factor: int = 1, train_image_names=None, scale: bool = True,
                 rotate: bool = True) -> dict:
    """{'image_names', 'camtoworlds' [N,4,4] f64, 'intrinsics' [N,3,3] f64, 'image_index_to_image_id', 'points3d',
    'colors', 'sizes' [N,2] (w,h of each image's camera / factor)} of a COLMAP binary model; scale / rotate:
    load_colmap's normalisation flags (its defaults, True)."""
    if factor not in (1, 2, 4, 8):
        raise ValueError(f"factor must be 1, 2, 4 or 8, got {factor}")
    m = SceneManager(colmap_dir, load_points=True)
    m.load()
    names, w2c, K, wh = [], [], [], []
    bottom = np.array([[0.0, 0.0, 0.0, 1.0]])
    for iid, im in m.images.items():
        if train_image_names and im.name not in train_image_names:
            continue
        names.append(im.name)
        cam = m.cameras[im.camera_id]
        K.append(np.array([[cam.fx / factor, 0, cam.cx / factor], [0, cam.fy / factor, cam.cy / factor], [0, 0, 1]]))
        w2c.append(np.concatenate([np.concatenate([im.R(), im.tvec.reshape(3, 1)], 1), bottom], 0))
        wh.append((cam.width // factor, cam.height // factor))
    if not names:
        raise ValueError(f"no images selected from {colmap_dir}")
    c2w = np.linalg.inv(np.stack(w2c))
    order = np.argsort(names)
    names = [names[i] for i in order]
    c2w, pts = c2w[order], m.points3D
    if scale:
        from .normalize import normalize_scene
        c2w, pts = normalize_scene(c2w, pts, scale=True, rotate=rotate)
        c2w, pts = np.asarray(c2w, dtype=np.float64), np.asarray(pts, dtype=np.float64)
    return {"image_names": names, "camtoworlds": c2w, "intrinsics": np.stack(K)[order],
            "sizes": np.asarray(wh, dtype=np.int64)[order],
            "image_index_to_image_id": {i: m.name_to_image_id[n] for i, n in enumerate(names)},
            "points3d": pts, "colors": m.point3D_colors}


def block_views(block_image_ids: dict, camtoworlds, intrinsics, image_paths, val_indices=()) -> dict:
    """load_colmap.py:459-487 -> {'poses': [c2w f32], 'intrinsics': [K f32], 'image_paths': [[path]]}, one entry per
    block, each block's members in image order with the validation images removed."""
    nb = len(block_image_ids)
    poses, Ks, paths = [None] * nb, [None] * nb, [None] * nb
    val = set(int(i) for i in np.asarray(val_indices).reshape(-1).tolist())
    c2w, K = np.asarray(camtoworlds), np.asarray(intrinsics)
    for b, ids in block_image_ids.items():
        members = set(int(i) for i in np.concatenate([np.asarray(x).reshape(-1) for x in ids]).tolist())
        sel = [i for i in range(len(image_paths)) if i in members and i not in val]
        if not sel:
            raise ValueError(f"block {b} has no training image")
        paths[b] = [image_paths[i] for i in sel]
        poses[b] = torch.from_numpy(c2w[sel]).float()
        Ks[b] = torch.from_numpy(K[sel]).float()
    return {"poses": poses, "intrinsics": Ks, "image_paths": paths}


@dataclass
class BlockCamera:
    """The fields Camera.compose_state_dict stores (geometry/camera.py:165-185)."""
    image_index: int
    width: int
    height: int
    world_to_camera: torch.Tensor     # [4,4] w2c (not transposed)
    fx: float
    fy: float
    cx: float
    cy: float
    image_path: str = ""

    def state_dict(self) -> dict:
        return {"world_to_camera": self.world_to_camera.detach().cpu().float(), "image_index": int(self.image_index),
                "width": int(self.width), "height": int(self.height), "image_path": self.image_path,
                "fx": float(self.fx), "fy": float(self.fy), "cx": float(self.cx), "cy": float(self.cy)}

    @classmethod
    def from_state_dict(cls, d: dict) -> "BlockCamera":
        return cls(d["image_index"], d["width"], d["height"], d["world_to_camera"], d["fx"], d["fy"], d["cx"],
                   d["cy"], d["image_path"])

    def raster_camera(self, device="cpu", znear: float = 0.01, zfar: float = 100.0) -> RasterCamera:
        return make_camera(self.width, self.height, self.fx, self.fy, self.world_to_camera, znear, zfar,
                           image_index=int(self.image_index)).to(device)


@dataclass
class MiniDataset:
    """dataset_base.py:96-150: one block's cameras and camera-to-world poses on disk."""
    cameras: list = field(default_factory=list)
    camtoworlds: torch.Tensor | None = None
    current_block: int = -1

    def __len__(self):
        return len(self.cameras)

    def write(self, path: str) -> None:
        cdir = os.path.join(path, "cameras")
        os.makedirs(cdir, exist_ok=True)
        for i, cam in enumerate(self.cameras):
            p = os.path.join(cdir, f"camera_{i}.pt")
            if not os.path.exists(p):            # as Camera.write: an existing file is kept
                torch.save(cam.state_dict(), p)
        p = os.path.join(path, "cameratoworlds.pt")
        if not os.path.exists(p):
            torch.save(self.camtoworlds, p)

    def read(self, path: str, block_id: int = 0, device="cpu") -> "MiniDataset":
        cdir = os.path.join(path, "cameras")
        files = sorted((f for f in os.listdir(cdir) if os.path.isfile(os.path.join(cdir, f))),
                       key=lambda f: int(f[len("camera_"):-len(".pt")]) if f.startswith("camera_") else -1)
        self.cameras = [BlockCamera.from_state_dict(torch.load(os.path.join(cdir, f), weights_only=True))
                        for f in files]
        self.camtoworlds = torch.load(os.path.join(path, "cameratoworlds.pt"), map_location=torch.device(device),
                                      weights_only=True)
        self.current_block = block_id
        return self


def export_blocks(out_dir: str, views: dict, block_image_ids: dict, image_paths=None, val_indices=()) -> list:
    """Writes out_dir/block_{k}/ (MiniDataset format) for each block of the split; returns the MiniDatasets."""
    paths = image_paths if image_paths is not None else views["image_names"]
    bv = block_views(block_image_ids, views["camtoworlds"], views["intrinsics"], paths, val_indices)
    index_of = {p: i for i, p in enumerate(paths)}
    out = []
    for b in range(len(block_image_ids)):
        cams = []
        for j, (c2w, K, p) in enumerate(zip(bv["poses"][b], bv["intrinsics"][b], bv["image_paths"][b])):
            w, h = (int(x) for x in views["sizes"][index_of[p]])
            # image_index: the camera's position in its block (compose_cameras, dataset_base.py:64-92, composes each
            # block's list with image_index = i; the appearance embedding and the exposure are indexed by it)
            cams.append(BlockCamera(j, w, h, torch.linalg.inv(c2w.double()).float(), float(K[0, 0]), float(K[1, 1]),
                                    float(K[0, 2]), float(K[1, 2]), p))
        ds = MiniDataset(cams, bv["poses"][b], b)
        ds.write(os.path.join(out_dir, f"block_{b}"))
        out.append(ds)
    return out
