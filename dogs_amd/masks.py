"""The decoupled appearance embedding of geometry.mask (VastGaussian's appearance CNN), as the reference trainers use it
(conerf/model/gaussian_fields/masks.py:8-54; gaussian_trainer.py:171-183 build, :232-235 its Adam, :392-401 the masked
loss, :482-484 the step).

The network is small and convolutional; on the GPU its 3x3 convolutions run on the library's kernels (Conv3x3:
dg_conv3x3 / dg_conv3x3_wgrad) and its full-resolution head on dg_mask_head_* (fixed-order sums, so the same bits in
every process), the rest is torch.  What the hot path needs from it is the [3, H, W] mask the photometric term
multiplies the render with.  The native training step (dg_train_step) takes that mask and returns
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
    return Conv3x3(cin, cout)


class Conv3x3(nn.Conv2d):
    """nn.Conv2d(cin, cout, 3, padding=1) -- the same parameters -- whose forward and backward on the GPU are the
    library's: dg_conv3x3 (the forward, and the input gradient as its adjoint) and dg_conv3x3_wgrad (weight and bias
    gradients), each a fixed-order sum with no atomics.  So the embedding is bitwise the same in every process: MIOpen
    picks its algorithm per process from its find database and what ran before (the masked ADMM ranks differed from the
    sequential baseline after other convolutions had run in the baseline's process, gpurun_out/det1), and its
    deterministic weight-gradient algorithm for the full-resolution convolutions took 83 ms per 1080p call."""

    def __init__(self, cin: int, cout: int) -> None:
        super().__init__(cin, cout, kernel_size=3, padding=1)

    def forward(self, x: torch.Tensor, relu: bool = False, shuffle: bool = False) -> torch.Tensor:
        """relu: max(conv(x), 0), the following nn.ReLU folded into the kernels (its backward too); shuffle: the
        convolution of pixel_shuffle(x, 2), the preceding nn.PixelShuffle(2) folded into the kernels' addressing."""
        if x.is_cuda:
            return _Conv3x3Fn.apply(x, self.weight, self.bias, relu, shuffle)
        y = super().forward(F.pixel_shuffle(x, 2) if shuffle else x)
        return F.relu(y) if relu else y


DG_CONV_ADJOINT, DG_CONV_RELU, DG_CONV_SHUFFLE = 1, 2, 4   # dg_conv3x3 flags (include/dogs_hip.h)


def _conv3x3(L, x4: torch.Tensor, w: torch.Tensor, b, out_chw: tuple, flags: int, gate=None) -> torch.Tensor:
    """dg_conv3x3 over each image of x4 [N, C, h, w] (float32, contiguous) into [N, *out_chw]; gate: [N, ...] like the
    output gradient or None.  H, W passed to the kernel are the convolution's (the larger side with the shuffle)."""
    from . import _lib
    n = int(x4.shape[0])
    H, W = (int(x4.shape[2]), int(x4.shape[3])) if not flags & DG_CONV_SHUFFLE or flags & DG_CONV_ADJOINT \
        else (2 * int(x4.shape[2]), 2 * int(x4.shape[3]))
    cin_w, cout_w = int(w.shape[1]), int(w.shape[0])
    y = torch.empty((n, *out_chw), dtype=torch.float32, device=x4.device)
    with _lib.device_ctx(x4.device):
        st = _lib.stream_of(x4.device)
        for i in range(n):
            _lib.check(L.dg_conv3x3(cin_w, cout_w, H, W, x4[i].data_ptr(), w.data_ptr(),
                                    b.data_ptr() if b is not None else None, y[i].data_ptr(), flags,
                                    gate[i].data_ptr() if gate is not None else None, st))
    return y


class _Conv3x3Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, relu=False, shuffle=False):
        from . import _lib
        if x.dtype != torch.float32 or weight.dtype != torch.float32:
            raise TypeError("Conv3x3 on the GPU takes float32")
        x4 = (x if x.dim() == 4 else x.unsqueeze(0)).contiguous()
        w = weight.contiguous()
        b = bias.contiguous() if bias is not None else None
        ctx.has_bias = bias is not None
        ctx.batched = x.dim() == 4
        ctx.shuffle = bool(shuffle)
        H, W = int(x4.shape[2]) * (2 if shuffle else 1), int(x4.shape[3]) * (2 if shuffle else 1)
        if shuffle and int(x4.shape[1]) != 4 * int(w.shape[1]):
            raise ValueError("Conv3x3 with shuffle takes 4 * in_channels input channels")
        flags = (DG_CONV_RELU if relu else 0) | (DG_CONV_SHUFFLE if shuffle else 0)
        y = _conv3x3(_lib.load(), x4, w, b, (int(w.shape[0]), H, W), flags)
        # with the ReLU folded in, its output gates the output gradient in both backward kernels
        ctx.save_for_backward(x4, w, y if relu else None)
        return y if ctx.batched else y[0]

    @staticmethod
    def backward(ctx, g):
        from . import _lib
        x4, w, gate = ctx.saved_tensors
        L = _lib.load()
        g4 = (g if g.dim() == 4 else g.unsqueeze(0)).contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            sh = DG_CONV_SHUFFLE if ctx.shuffle else 0
            dx = _conv3x3(L, g4, w, None, tuple(int(v) for v in x4.shape[1:]), DG_CONV_ADJOINT | sh, gate)
            dx = dx if ctx.batched else dx[0]
        dw = db = None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            cout, cin = int(w.shape[0]), int(w.shape[1])
            dw = torch.empty_like(w)
            db = torch.empty(cout, dtype=torch.float32, device=w.device)
            for b in range(int(x4.shape[0])):    # one image per call, summed in batch order
                H, W = int(g4.shape[2]), int(g4.shape[3])
                nbytes = int(L.dg_conv3x3_wgrad_scratch_bytes(cin, cout, H, W))
                scratch = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=w.device)
                dwb, dbb = (dw, db) if b == 0 else (torch.empty_like(dw), torch.empty_like(db))
                with _lib.device_ctx(w.device):
                    _lib.check(L.dg_conv3x3_wgrad(cin, cout, H, W, x4[b].data_ptr(), g4[b].data_ptr(),
                                                  gate[b].data_ptr() if gate is not None else None,
                                                  DG_CONV_SHUFFLE if ctx.shuffle else 0, dwb.data_ptr(),
                                                  dbb.data_ptr(), scratch.data_ptr(), nbytes,
                                                  _lib.stream_of(w.device)))
                if b:
                    dw += dwb
                    db += dbb
        return dx, dw, (db if ctx.has_bias else None), None, None


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
        x = self.fusion(x)
        for st in self.upsample:   # (PixelShuffle, Conv3x3, ReLU): shuffle and ReLU folded into the convolution's kernels
            x = st[1](x, relu=True, shuffle=True)
        H, W = int(image_size[0]), int(image_size[1])
        if x.is_cuda and x.dim() == 3 and H <= 4 * x.shape[1] and W <= 4 * x.shape[2]:
            c1, c2 = self.out_conv[0], self.out_conv[2]
            return _MaskHead.apply(x, c1.weight, c1.bias, c2.weight, c2.bias, (H, W))
        x = resize_bilinear(x, (H, W))
        return self.out_conv(x)


class _MaskHead(torch.autograd.Function):
    """The full-resolution head resize -> out_conv (Conv2d 16 -> 8, ReLU, Conv2d 8 -> 3) as dg_mask_head_forward /
    dg_mask_head_backward (mask_head.hip): the 16-channel full-size image is never materialised, and the backward's
    sums run in a fixed order (deterministic, no atomics).  The same function as the torch modules (fp32 rounding
    differs: tests/test_gpu_mask_conv.py)."""

    @staticmethod
    def forward(ctx, u, w1, b1, w2, b2, size):
        from . import _lib
        H, W = size
        uc = u.detach().contiguous()
        ps = [t.detach().contiguous() for t in (w1, b1, w2, b2)]
        mask = torch.empty((3, H, W), dtype=torch.float32, device=u.device)
        # the hidden layer, kept for the backward when one will run (it then skips the samples and conv1)
        hid = torch.empty((8, H, W), dtype=torch.float32, device=u.device) if any(ctx.needs_input_grad) else None
        with _lib.device_ctx(u.device):
            _lib.check(_lib.load().dg_mask_head_forward(H, W, int(uc.shape[1]), int(uc.shape[2]), uc.data_ptr(),
                                                        *[p.data_ptr() for p in ps], mask.data_ptr(),
                                                        hid.data_ptr() if hid is not None else None,
                                                        _lib.stream_of(u.device)))
        ctx.hid = hid
        ctx.save_for_backward(uc, *ps)
        ctx.size = (H, W)
        return mask

    @staticmethod
    def backward(ctx, g):
        from . import _lib
        uc, w1, b1, w2, b2 = ctx.saved_tensors
        H, W = ctx.size
        L = _lib.load()
        gc = g.contiguous()
        du = torch.empty_like(uc)
        npar = int(L.dg_mask_head_nparams())
        dp = torch.empty(npar, dtype=torch.float32, device=uc.device)
        nbytes = int(L.dg_mask_head_scratch_bytes(H, W))
        scratch = torch.empty(nbytes, dtype=torch.uint8, device=uc.device)
        with _lib.device_ctx(uc.device):
            hid = ctx.hid
            _lib.check(L.dg_mask_head_backward(H, W, int(uc.shape[1]), int(uc.shape[2]), uc.data_ptr(),
                                               w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(),
                                               gc.data_ptr(), hid.data_ptr() if hid is not None else None,
                                               du.data_ptr(), dp.data_ptr(), scratch.data_ptr(), nbytes,
                                               _lib.stream_of(uc.device)))
        ctx.hid = None
        n1, n2 = w1.numel(), w2.numel()
        dw1, db1 = dp[:n1].view_as(w1), dp[n1:n1 + b1.numel()]
        o = n1 + b1.numel()
        dw2, db2 = dp[o:o + n2].view_as(w2), dp[o + n2:o + n2 + b2.numel()]
        return du, dw1, db1, dw2, db2, None


def _bilinear_taps(n_in: int, n_out: int, device) -> tuple:
    """Per output index: (i0, i1, l0, l1) of upsample_bilinear2d with align_corners=False and a given size (torch's
    area_pixel_compute_source_index: src = (dst + 0.5) in / out - 0.5 clamped at 0, float32 arithmetic)."""
    scale = torch.tensor(n_in / n_out, dtype=torch.float32)
    dst = torch.arange(n_out, dtype=torch.float32)
    src = torch.clamp_min(scale * (dst + 0.5) - 0.5, 0.0)
    i0 = src.to(torch.int64)
    i1 = torch.clamp_max(i0 + 1, n_in - 1)
    l1 = src - i0.to(torch.float32)
    l0 = 1.0 - l1
    return i0, i1, l0, l1


_ADJ_CACHE: dict = {}


def _adjoint_gather(n_in: int, n_out: int, device) -> tuple:
    """(idx [n_in, L], wt [n_in, L]): every output index that reads input index i, with its weight, in ascending output
    order (zero-weight padding).  The adjoint of the resize along one axis is then a gather, a product and a sum over L
    in a fixed order -- no atomics."""
    key = (n_in, n_out, str(device))
    hit = _ADJ_CACHE.get(key)
    if hit is not None:
        return hit
    i0, i1, l0, l1 = _bilinear_taps(n_in, n_out, "cpu")
    taps = [[] for _ in range(n_in)]
    for o in range(n_out):
        a, b = int(i0[o]), int(i1[o])
        taps[a].append((o, float(l0[o])))
        taps[b].append((o, float(l1[o])))      # a == b at the clamped edge: two taps of the same output
    L = max(1, max(len(t) for t in taps))
    idx = torch.zeros((n_in, L), dtype=torch.int64)
    wt = torch.zeros((n_in, L), dtype=torch.float32)
    for i, t in enumerate(taps):
        t.sort(key=lambda ow: ow[0])
        for k, (o, w) in enumerate(t):
            idx[i, k], wt[i, k] = o, w
    hit = _ADJ_CACHE[key] = (idx.to(device), wt.to(device))
    return hit


class _ResizeBilinear(torch.autograd.Function):
    """F.interpolate(mode="bilinear") forward (the reference module's values, bit for bit) with a deterministic
    backward: torch's upsample_bilinear2d backward scatters with atomicAdd on the GPU, so two runs of a masked
    training loop (or the ranks and the sequential baseline of an ADMM run) drift apart by rounding.  Here the adjoint
    runs as two gathers along W, then H, each summing its taps in a fixed order."""

    @staticmethod
    def forward(ctx, x, size):
        ctx.in_hw = (int(x.shape[-2]), int(x.shape[-1]))
        return F.interpolate(x.unsqueeze(0), size=size, mode="bilinear")[0]

    @staticmethod
    def backward(ctx, g):
        h, w = ctx.in_hw
        H, W = int(g.shape[-2]), int(g.shape[-1])
        iw, ww = _adjoint_gather(w, W, g.device)
        gw = (g[:, :, iw] * ww).sum(-1)                        # [C, H, w]
        ih, wh = _adjoint_gather(h, H, g.device)
        gx = (gw[:, ih, :] * wh[:, :, None]).sum(-2)           # [C, h, w]
        return gx, None


def resize_bilinear(x: torch.Tensor, size: tuple) -> torch.Tensor:
    """[C, h, w] -> [C, H, W] bilinear (align_corners=False), deterministic backward (_ResizeBilinear)."""
    return _ResizeBilinear.apply(x, size)


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
