"""numpy restatement of the reference's read_image -- TEST INFRASTRUCTURE ONLY (imported only by tests/).

conerf/base/task_queue.py:13-27: torch.from_numpy(imread(path)).to(uint8); (image / 255.0).clamp(0, 1) in float32;
RGBA: image[..., :3] * image[..., 3:4] + np.array([0, 0, 0]) * (1 - image[..., 3:4]) -- numpy float32 with an int64
background, so float64 -- then .float().  The decode itself (imageio) is not restated: the input is the decoded
u8 array.
"""
from __future__ import annotations

import numpy as np


def read_image(u8: np.ndarray, num_channels: int = 3) -> np.ndarray:
    img = np.clip(u8.astype(np.float32) / np.float32(255.0), 0.0, 1.0).astype(np.float32)
    if img.ndim == 2:
        img = img[:, :, None]
    if num_channels == 4 and img.shape[2] == 4:
        background = np.array([0, 0, 0])
        img = img[:, :, :3] * img[:, :, 3:4] + background * (1 - img[:, :, 3:4])
        img = img.astype(np.float32)
    return img
