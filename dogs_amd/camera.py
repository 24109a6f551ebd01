"""Camera matrices in the reference's conventions.

Restates conerf/geometry/camera.py:79-135 (focal_length_to_fov, Camera.__init__) and
conerf/geometry/pose_util.py:428-448 (projection_matrix): the rasterizer receives
viewmatrix = w2c^T, projmatrix = w2c^T @ P^T (row-vector convention) and
campos = inverse(w2c^T)[3, :3].  The principal point is ignored by the rasterizer.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch


def focal_length_to_fov(focal_length: float, pixels: int) -> float:
    return 2 * math.atan(pixels / (2 * focal_length))


def projection_matrix(znear: float, zfar: float, fov_x: float, fov_y: float) -> torch.Tensor:
    tan_half_fov_y = math.tan(fov_y / 2)
    tan_half_fov_x = math.tan(fov_x / 2)
    top = tan_half_fov_y * znear
    bottom = -top
    right = tan_half_fov_x * znear
    left = -right
    P = torch.zeros(4, 4)
    z_sign = 1.0
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = z_sign
    P[2, 2] = z_sign * zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


@dataclass
class RasterCamera:
    width: int
    height: int
    fov_x: float
    fov_y: float
    world_to_camera: torch.Tensor      # [4,4] = w2c^T (what the rasterizer calls viewmatrix)
    projective_matrix: torch.Tensor    # [4,4] = w2c^T @ P^T
    camera_center: torch.Tensor        # [3]
    image_index: int = -1              # the dataset's image index (appearance embedding / trained exposure row)
    znear: float = 0.01
    zfar: float = 100.0

    @property
    def tanfovx(self) -> float:
        return math.tan(self.fov_x * 0.5)

    @property
    def tanfovy(self) -> float:
        return math.tan(self.fov_y * 0.5)

    def to(self, device) -> "RasterCamera":
        return RasterCamera(self.width, self.height, self.fov_x, self.fov_y,
                            self.world_to_camera.to(device), self.projective_matrix.to(device),
                            self.camera_center.to(device), self.image_index, self.znear, self.zfar)

    @property
    def fx(self) -> float:
        return self.width / (2.0 * math.tan(self.fov_x * 0.5))

    @property
    def fy(self) -> float:
        return self.height / (2.0 * math.tan(self.fov_y * 0.5))

    def downsample(self, resolution: int = 1) -> "RasterCamera":
        """Camera.downsample (conerf/geometry/camera.py:146-163): focal lengths / resolution, image size
        ceil(size / resolution), the same pose; the matrices are rebuilt on the camera's device."""
        if resolution == 1:
            return self
        dev = self.world_to_camera.device
        w2c = self.world_to_camera.detach().cpu().transpose(0, 1)
        cam = make_camera(math.ceil(self.width / resolution), math.ceil(self.height / resolution),
                          self.fx / resolution, self.fy / resolution, world_to_camera=w2c, znear=self.znear,
                          zfar=self.zfar)
        cam.image_index = self.image_index
        return cam.to(dev)


def make_camera(width: int, height: int, fx: float, fy: float, world_to_camera: torch.Tensor | None = None,
                znear: float = 0.01, zfar: float = 100.0, image_index: int = -1) -> RasterCamera:
    if world_to_camera is None:
        world_to_camera = torch.eye(4)
    w2c = world_to_camera.to(torch.float32)
    fov_x = focal_length_to_fov(fx, width)
    fov_y = focal_length_to_fov(fy, height)
    view = w2c.clone().transpose(0, 1)
    proj = projection_matrix(znear, zfar, fov_x, fov_y).transpose(0, 1)
    full = view @ proj
    center = view.inverse()[3, :3]
    return RasterCamera(width, height, fov_x, fov_y, view.contiguous(), full.contiguous(), center.contiguous(),
                        image_index, znear, zfar)


def yaw_world_to_camera(yaw_rad: float) -> torch.Tensor:
    """Camera at the origin rotated about +y by yaw (used to build seeded view batches)."""
    c, s = math.cos(yaw_rad), math.sin(yaw_rad)
    w2c = torch.eye(4)
    w2c[0, 0], w2c[0, 2], w2c[2, 0], w2c[2, 2] = c, -s, s, c
    return w2c
