"""Synthetic scenes of BASELINE.md §2 / SURVEY.md §8(d).

Drawn on the CPU with torch.Generator().manual_seed(seed) in a fixed order:
z ~ U[2,20]; x = U[-1,1]*z*(W/2fx)*1.1; y = U[-1,1]*z*(H/2fy)*1.1; log-scale ~ N(ln 0.02, 0.5)^3;
raw quaternion ~ N(0,1)^4 (normalised like GaussianSplatModel.get_quaternion);
raw opacity ~ N(0,1.5) -> sigmoid; dc ~ N(0,0.3); rest ~ N(0,0.05).
The camera is world_to_camera = I, fx = fy = 1600 (1080p; 800x800 and 4K variants by size).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from .camera import RasterCamera, make_camera


@dataclass
class SyntheticScene:
    means3D: torch.Tensor      # [N,3]
    scales: torch.Tensor       # [N,3] activated (exp)
    rotations: torch.Tensor    # [N,4] normalised
    opacities: torch.Tensor    # [N,1] activated (sigmoid)
    dc: torch.Tensor           # [N,1,3]
    sh: torch.Tensor           # [N,15,3]
    raw_scales: torch.Tensor
    raw_rotations: torch.Tensor
    raw_opacities: torch.Tensor
    camera: RasterCamera

    def to(self, device) -> "SyntheticScene":
        f = lambda t: t.to(device)
        return SyntheticScene(f(self.means3D), f(self.scales), f(self.rotations), f(self.opacities), f(self.dc),
                              f(self.sh), f(self.raw_scales), f(self.raw_rotations), f(self.raw_opacities),
                              self.camera.to(device))

    @property
    def n(self) -> int:
        return self.means3D.shape[0]


def make_scene(n: int, width: int = 1920, height: int = 1080, fx: float = 1600.0, fy: float = 1600.0,
               seed: int = 1234, sh_rest: int = 15, opacity_mean: float = 0.0) -> SyntheticScene:
    """opacity_mean shifts the raw opacity (N(opacity_mean, 1.5)): the default 0 is BASELINE §2's scene, where near
    Gaussians saturate almost every tile; -2 is the bench's non-saturating variant (most tiles see their whole list)."""
    g = torch.Generator().manual_seed(seed)
    z = torch.empty(n).uniform_(2.0, 20.0, generator=g)
    ux = torch.empty(n).uniform_(-1.0, 1.0, generator=g)
    uy = torch.empty(n).uniform_(-1.0, 1.0, generator=g)
    x = ux * z * (width / (2 * fx)) * 1.1
    y = uy * z * (height / (2 * fy)) * 1.1
    means = torch.stack([x, y, z], dim=1).contiguous()
    raw_s = torch.randn(n, 3, generator=g) * 0.5 + math.log(0.02)
    raw_q = torch.randn(n, 4, generator=g)
    raw_o = torch.randn(n, 1, generator=g) * 1.5
    if opacity_mean != 0.0:
        raw_o = raw_o + opacity_mean
    dc = torch.randn(n, 1, 3, generator=g) * 0.3
    sh = torch.randn(n, sh_rest, 3, generator=g) * 0.05
    scales = torch.exp(raw_s)
    rot = torch.nn.functional.normalize(raw_q)
    opac = torch.sigmoid(raw_o)
    cam = make_camera(width, height, fx, fy)
    return SyntheticScene(means, scales.contiguous(), rot.contiguous(), opac.contiguous(), dc.contiguous(),
                          sh.contiguous(), raw_s, raw_q, raw_o, cam)
