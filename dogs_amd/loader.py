"""The training image path, drop-in for conerf/base/task_queue.py:

* `read_image(path, num_channels)` -- task_queue.py:13-27: a float32 HWC image in [0, 1] (with num_channels == 4,
  RGBA composited over black); here on the GPU (`device`), from the image's decoded u8 cache.
* `ImageReader(max_size, max_num_threads, num_channels, image_list)` -- task_queue.py:89-152 with the same methods
  (`add_task(None)`, `get_image()`, `num_images()`, `safe_exit()`).  Its images come from a native ring
  (`dg_ring_*`): C++ reader threads fill pinned slots with u8 bytes, and `get_image` uploads them with an async copy
  on the current stream and converts them to float on the GPU -- a quarter of the PCIe bytes of the reference's
  float copy and no host wait.  `get_image` returns the HWC float view of a CHW device tensor, so the trainer's
  `camera.image.permute(2, 0, 1)` is the contiguous CHW image (`copy_to_device` is then a no-op).

Decoded cache: an image path `x.png` is read from `x.png.npy` (u8 HWC, written once by `decode_to_cache` with
Pillow) or the path itself when it is a `.npy` file; the ring never decodes.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch

from . import _lib


def cache_path(image_path: str) -> str:
    return image_path if image_path.endswith(".npy") else image_path + ".npy"


def decode_to_cache(image_path: str) -> str:
    """One-time decode of a PNG/JPEG into its u8 HWC .npy cache (Pillow; the reference decodes with imageio)."""
    out = cache_path(image_path)
    if not os.path.exists(out):
        from PIL import Image
        with Image.open(image_path) as im:
            arr = np.asarray(im)
        if arr.dtype != np.uint8:
            raise ValueError(f"{image_path}: only 8-bit images are supported")
        np.save(out, arr if arr.ndim == 3 else arr[:, :, None])
    return out


def _npy_layout(path: str):
    """(data offset, h, w, c) of a u8 .npy file, from its header (no data read)."""
    with open(path, "rb") as f:
        version = np.lib.format.read_magic(f)
        read = np.lib.format.read_array_header_1_0 if version == (1, 0) else np.lib.format.read_array_header_2_0
        shape, fortran, dtype = read(f)
        offset = f.tell()
    if dtype != np.uint8 or fortran or len(shape) not in (2, 3):
        raise ValueError(f"{path}: expected a C-order u8 HxW[xC] array")
    h, w = int(shape[0]), int(shape[1])
    c = int(shape[2]) if len(shape) == 3 else 1
    return offset, h, w, c


class ImageReader:
    """task_queue.py:89-152 over the native pinned ring."""

    def __init__(self, max_size: int = 100, max_num_threads: int = 8, num_channels: int = 3, image_list=None,
                 device=None, max_image_bytes: int | None = None):
        self.image_list = list(image_list or [])
        self.num_channels = num_channels
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self._layout = [_npy_layout(cache_path(p)) for p in self.image_list]
        max_bytes = max_image_bytes or max([h * w * c for _, h, w, c in self._layout] or [1])
        self._slots = max(2, min(int(max_size), len(self.image_list) or 2))
        self._L = _lib.load()
        self._ring = self._L.dg_ring_create(self._slots, int(max_bytes), int(max_num_threads))
        if not self._ring:
            raise RuntimeError("dg_ring_create failed (pinned host memory)")
        self._staging = torch.empty(int(max_bytes), dtype=torch.uint8, device=self.device)
        self._outstanding = 0

    def add_task(self, task=None, *args, **kwargs):  # noqa: ARG002 - the reference's signature
        for i, p in enumerate(self.image_list):
            off, h, w, c = self._layout[i]
            rc = self._L.dg_ring_submit(self._ring, cache_path(p).encode(), off, i, h, w, c)
            if rc:
                raise RuntimeError(f"dg_ring_submit({p}) failed ({rc})")
            self._outstanding += 1

    def get_image(self):
        """(index, float32 HWC image on the device) in completion order."""
        idx, h, w, c, slot = C.c_int(), C.c_int(), C.c_int(), C.c_int(), C.c_int()
        rc = self._L.dg_ring_next(self._ring, C.byref(idx), C.byref(h), C.byref(w), C.byref(c), C.byref(slot))
        self._outstanding -= 1
        if rc:
            raise RuntimeError(f"image {idx.value}: read failed")
        H, W, Cin = h.value, w.value, c.value
        composite = int(self.num_channels == 4 and Cin == 4)
        out = torch.empty((3 if composite else Cin, H, W), dtype=torch.float32, device=self.device)
        with _lib.device_ctx(self.device):
            rc = self._L.dg_ring_upload(self._ring, slot.value, H, W, Cin, composite, self._staging.data_ptr(),
                                        out.data_ptr(), _lib.stream_of(self.device))
        if rc:
            raise RuntimeError(f"dg_ring_upload failed ({rc})")
        return idx.value, out.permute(1, 2, 0)

    def num_images(self) -> int:
        return self._outstanding

    def safe_exit(self):
        while self._outstanding > 0:
            self.get_image()
        self.close()

    def close(self):
        if getattr(self, "_ring", None):
            torch.cuda.synchronize(self.device)
            self._L.dg_ring_destroy(self._ring)
            self._ring = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def read_image(image_path: str, num_channels: int = 3, device=None) -> torch.Tensor:
    """task_queue.py:13-27 on the GPU: float32 HWC in [0, 1] from the decoded cache."""
    arr = np.load(cache_path(image_path), mmap_mode="r")
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    u8 = torch.from_numpy(np.ascontiguousarray(arr)).to(dev)
    H, W = u8.shape[0], u8.shape[1]
    Cin = u8.shape[2] if u8.dim() == 3 else 1
    composite = int(num_channels == 4 and Cin == 4)
    out = torch.empty((3 if composite else Cin, H, W), dtype=torch.float32, device=dev)
    with _lib.device_ctx(dev):
        _lib.check(_lib.load().dg_image_u8_to_chw(u8.data_ptr(), H, W, Cin, composite, out.data_ptr(),
                                                  _lib.stream_of(dev)))
    return out.permute(1, 2, 0)
