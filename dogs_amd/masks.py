"""The decoupled appearance embedding of geometry.mask (VastGaussian's appearance CNN), as the reference trainers use it
(conerf/model/gaussian_fields/masks.py:8-54; gaussian_trainer.py:171-183 build, :232-235 its Adam, :392-401 the masked
loss, :482-484 the step).

The network is small and convolutional -- torch (MIOpen) runs it; what the hot path needs from it is the [3, H, W] mask
the photometric term multiplies the render with.  The native training step (dg_train_step) takes that mask and returns
dL/dmask, and the trainer back-propagates it through this module (`MaskedStep`).

Parameter names and shapes follow the reference module, so its state dicts load unchanged: `appearance_embedding`
[num_views, 64], `fusion` (3x3 conv, 67 -> 256), `upsample.{0..3}` = (PixelShuffle(2), 3x3 conv c/4 -> c/2, ReLU) for
c = 256, 128, 64, 32, then `out_conv` = (3x3 conv 16 -> 8, ReLU, 3x3 conv 8 -> 3).  Forward: the low-resolution target
(the camera downsampled 32x) concatenated with the view's embedding, fused, upsampled 16x by the four shuffle stages,
bilinearly resized to the full image size, and mapped to three channels without a final activation.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F
from torch import nn

EMBEDDING_DIM = 64
MASK_DOWNSAMPLE = 32          # camera_origin.downsample(32) (gaussian_trainer.py:394)
_STAGE_CHANNELS = (256, 128, 64, 32)


def _conv3(cin: int, cout: int) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, kernel_size=3, padding=1)


class AppearanceEmbedding(nn.Module):
    def __init__(self, num_views: int, embedding_dim: int = EMBEDDING_DIM) -> None:
        super().__init__()
        self.appearance_embedding = nn.Parameter(torch.zeros(num_views, embedding_dim))
        self.fusion = _conv3(embedding_dim + 3, _STAGE_CHANNELS[0])
        stages = []
        for c in _STAGE_CHANNELS:   # PixelShuffle(2) divides the channels by 4, the conv doubles them back to c / 2
            stages.append(nn.Sequential(nn.PixelShuffle(2), _conv3(c // 4, c // 2), nn.ReLU()))
        self.upsample = nn.Sequential(*stages)
        self.out_conv = nn.Sequential(_conv3(_STAGE_CHANNELS[-1] // 2, 8), nn.ReLU(), _conv3(8, 3))

    def forward(self, image: torch.Tensor, index: int, image_size: tuple) -> torch.Tensor:
        """image: [3, h, w] (the 32x-downsampled target); index: the view's row of the embedding table;
        image_size: (H, W) of the render.  Returns the [3, H, W] mask."""
        _, h, w = image.shape
        code = self.appearance_embedding[index]
        x = torch.cat([image, code[:, None, None].expand(code.shape[0], h, w)], dim=0)
        x = self.upsample(self.fusion(x))
        x = F.interpolate(x.unsqueeze(0), size=tuple(image_size), mode="bilinear")[0]
        return self.out_conv(x)


def downsample_image(image: torch.Tensor, factor: int) -> torch.Tensor:
    """The image of Camera.downsample(factor) (conerf/geometry/camera.py:146-163): [3, H, W] ->
    [3, ceil(H / factor), ceil(W / factor)] through torchvision's Resize as the pinned torchvision 0.15.2 applies it
    to a float tensor (bilinear, half-pixel centres, no antialiasing).  factor 1 returns the image itself."""
    if factor == 1:
        return image
    _, H, W = image.shape
    size = (math.ceil(H / factor), math.ceil(W / factor))
    return F.interpolate(image.unsqueeze(0), size=size, mode="bilinear", align_corners=False, antialias=False)[0]


class MaskedStep:
    """The trainer side of a native step with the appearance mask: evaluates the mask before the step (it depends only
    on the target and the view's embedding), hands dg_train_step the mask and a dL/dmask buffer, then runs the
    network's backward and its Adam step (gaussian_trainer.py:482-484).  `small` caches the 32x-downsampled targets."""

    def __init__(self, net: AppearanceEmbedding, optimizer: torch.optim.Optimizer):
        self.net, self.opt = net, optimizer
        self.small: dict = {}
        self.mask = None
        self.dmask: dict = {}

    def small_target(self, k: int, gt: torch.Tensor) -> torch.Tensor:
        t = self.small.get(k)
        if t is None:
            t = self.small[k] = downsample_image(gt, MASK_DOWNSAMPLE).contiguous()
        return t

    def forward(self, k: int, gt: torch.Tensor, index: int) -> tuple:
        """(mask [3,H,W] contiguous, dmask buffer of the same shape) for view k."""
        H, W = int(gt.shape[1]), int(gt.shape[2])
        self.mask = self.net(self.small_target(k, gt), index, (H, W))
        buf = self.dmask.get((H, W))
        if buf is None:
            buf = self.dmask[(H, W)] = torch.empty((3, H, W), dtype=torch.float32, device=gt.device)
        m = self.mask.detach()
        if not m.is_contiguous():
            m = m.contiguous()
        self._m = m
        return m, buf

    def backward_and_step(self, dmask: torch.Tensor) -> None:
        self.mask.backward(dmask)
        self.opt.step()
        self.opt.zero_grad(set_to_none=True)
        self.mask = self._m = None
