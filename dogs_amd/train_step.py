"""The native training step (dg_train_step): one GaussianSplatTrainer.train_iteration after densify_end_iter
(gaussian_trainer.py:324-476) -- activations, rasterizer forward, render()'s clamp + L1, fused SSIM, the loss
gradient, rasterizer backward, the scale regulariser, activation backward and SparseGaussianAdam (with an ADMM block
trainer's proximal gradient and the densification statistics when given) -- as one C call.

It runs the kernels of the autograd route with the same arithmetic (tests/test_gpu_admm.py compares the two), but
the host issues ~15 launches after the forward's one wait instead of ~100 Python-level operations, so the GPU does
not wait for the host between views.  The per-view argument blocks are built once; a step rewrites only the view's
learning rate, the proximal pointers and the depth-prefix policy."""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib

# setup_optimizer's group order (gaussian_trainer.py:205-230), which dg_train_step_args.groups follows
C_ORDER = ("xyz", "features_dc", "features_rest", "opacity", "scaling", "quaternion")
GROUP_NAME = {"xyz": "xyz", "features_dc": "f_dc", "features_rest": "f_rest", "opacity": "opacity",
              "scaling": "scaling", "quaternion": "quaternion"}


class NativeTrainStep:
    """params: {name: leaf tensor} for the six raw tensors (C_ORDER names); opt: the SparseGaussianAdam holding them
    (its exp_avg / exp_avg_sq state is created here when absent, the tensors the autograd route would create);
    cameras / images: the views (dogs_amd.camera.RasterCamera on the device, [3,H,W] targets); stats (optional):
    {max_radii2D, grad_accum, denom} updated each step (gaussian_trainer.py:433-438)."""

    def __init__(self, params: dict, opt, cameras: list, images: list, sh_degree: int, lambda_dssim: float,
                 lambda_scale: float, bg: torch.Tensor, device: torch.device, stats: dict | None = None,
                 overlap: bool = False, lambda_mask: float = 0.0, depth_threshold: float = 0.0,
                 antialiasing: bool = False):
        """lambda_mask: loss.lambda_mask (used by steps given a mask); depth_threshold: geometry.depth_threshold (scales
        the screen-space gradient the densification statistics read); antialiasing: texture.anti_aliasing."""
        self.L = _lib.load()
        self.device = device
        self.lambda_mask = float(lambda_mask)
        self.depth_threshold = float(depth_threshold or 0.0)
        self.antialiasing = bool(antialiasing)
        # overlap: each step returns with its f_dc / f_rest update still running on a side stream; the next step waits
        # for it before its binning emission (the first launch reading them) -- call sync() before anything else
        # touches those tensors or their Adam moments (rebind() does)
        self.overlap = bool(overlap) and hasattr(self.L, "dg_train_sync")
        self.arena = _lib.ReuseArena(device, keep_retired=self.overlap)
        self.lambdas = (float(lambda_dssim), float(lambda_scale))
        self.sh_degree = int(sh_degree)
        self.loss_buf = torch.zeros(4, dtype=torch.float32, device=device)
        self.last_masked = False
        self.bg = bg.to(device=device, dtype=torch.float32).contiguous()
        self.cameras, self.gt_images = cameras, images
        for cam, gt in zip(cameras, images):
            for t in (cam.world_to_camera, cam.projective_matrix, cam.camera_center, gt):
                if not (t.is_contiguous() and t.dtype == torch.float32 and t.device == device):
                    raise RuntimeError("native step: cameras and targets must be contiguous float32 on the device")
        self.images_out = {}
        self.opt = opt
        self.stream = _lib.stream_of(device)
        self.last_view = None
        self.rebind(params, stats)

    def rebind(self, params: dict | None = None, stats: dict | None = None) -> None:
        """(Re)build the argument blocks from the current tensors: after densify_and_prune, reset_opacity, a prune or
        optimizer.load_state_dict replaced the parameters or their Adam moments.  params: {C_ORDER name: tensor}
        (None: the optimizer's current group tensors); stats: the densification statistics (None: none)."""
        self.sync()
        opt, device = self.opt, self.device
        groups = {g["name"]: g for g in opt.param_groups}
        if params is None:
            params = {n: groups[GROUP_NAME[n]]["params"][0] for n in C_ORDER}
        P = int(params["xyz"].shape[0])
        rest = params["features_rest"]
        M = int(rest.shape[1]) if rest.dim() == 3 else 0
        self.params = params
        self.radii = torch.zeros(P, dtype=torch.int32, device=device)
        self.sh_status = torch.zeros(P, dtype=torch.uint8, device=device) if self.overlap else None
        for n in C_ORDER:
            p = params[n]
            if not (p.is_contiguous() and p.dtype == torch.float32 and p.device == device):
                raise RuntimeError(f"native step: {n} must be a contiguous float32 tensor on {device}")
            if int(p.shape[0]) != P:
                raise RuntimeError(f"native step: {n} has {int(p.shape[0])} rows, xyz {P}")
            if groups[GROUP_NAME[n]]["params"][0] is not p:
                raise RuntimeError(f"native step: {n} is not the tensor the optimizer's '{GROUP_NAME[n]}' group holds")
            st = opt.state[p]
            if len(st) == 0:
                st["step"] = torch.tensor(0.0, dtype=torch.float32)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        self.stats = None
        self.keep = [self.bg, self.cameras, self.gt_images]
        if stats is not None:
            for k in ("max_radii2D", "grad_accum", "denom"):
                t = stats[k]
                if not (t.is_contiguous() and t.dtype == torch.float32 and t.device == device and t.numel() == P):
                    raise RuntimeError(f"native step: {k} must be a contiguous float32 tensor of {P} on {device}")
            self.stats = _lib.DgDensifyStats(None, None, 3, stats["max_radii2D"].data_ptr(),
                                             stats["grad_accum"].data_ptr(), stats["denom"].data_ptr())
            self.keep.append(stats)
        # what the argument blocks point at: checked by every step (a replaced tensor would be a use-after-free)
        self._bound = self._pointers()
        self.args = []
        for cam, gt in zip(self.cameras, self.gt_images):
            a = _lib.DgTrainStepArgs()
            v = a.view
            v.P, v.D, v.M, v.W, v.H = P, self.sh_degree, M, int(cam.width), int(cam.height)
            v.prefiltered, v.antialiasing, v.debug = 0, int(self.antialiasing), 0
            v.scale_modifier, v.tanfovx, v.tanfovy = 1.0, float(cam.tanfovx), float(cam.tanfovy)
            v.bg, v.viewmatrix = self.bg.data_ptr(), cam.world_to_camera.data_ptr()
            v.projmatrix, v.campos = cam.projective_matrix.data_ptr(), cam.camera_center.data_ptr()
            a.gt = gt.data_ptr()
            a.lambda_dssim, a.lambda_scale = self.lambdas
            a.lambda_mask, a.depth_threshold = self.lambda_mask, self.depth_threshold
            for i, n in enumerate(C_ORDER):
                p = params[n]
                st = opt.state[p]
                g = groups[GROUP_NAME[n]]
                a.groups[i] = _lib.DgAdamGroup(p.data_ptr(), None, st["exp_avg"].data_ptr(),
                                               st["exp_avg_sq"].data_ptr(), float(g["lr"]), float(g["eps"]),
                                               int(p.numel() // P) if P else 1)
            key = (int(cam.height), int(cam.width))
            if key not in self.images_out:
                self.images_out[key] = torch.empty((3, key[0], key[1]), dtype=torch.float32, device=device)
            a.radii, a.image, a.loss = self.radii.data_ptr(), self.images_out[key].data_ptr(), self.loss_buf.data_ptr()
            a.stats = C.addressof(self.stats) if self.stats is not None else None
            a.sh_status = self.sh_status.data_ptr() if self.sh_status is not None else None
            self.args.append(a)

    def _pointers(self) -> tuple:
        """(param, exp_avg, exp_avg_sq) data pointers of the optimizer's current group tensors, C_ORDER."""
        groups = {g["name"]: g for g in self.opt.param_groups}
        out = []
        for n in C_ORDER:
            p = groups[GROUP_NAME[n]]["params"][0]
            st = self.opt.state.get(p, {})
            m, v = st.get("exp_avg"), st.get("exp_avg_sq")
            out.append((p.data_ptr(), m.data_ptr() if m is not None else 0, v.data_ptr() if v is not None else 0,
                        int(p.shape[0])))
        return tuple(out)

    def step(self, k: int, xyz_lr: float | None = None, prox: dict | None = None, sh_degree: int | None = None,
             lrs: dict | None = None, mask: torch.Tensor | None = None, dmask: torch.Tensor | None = None) -> None:
        """One iteration on view k; prox: {group name: (u, z, coef)} (ADMMBlockState.prox) or None; sh_degree: the
        model's active SH degree (increase_SH_degree), default the constructor's; lrs: {group name: lr} overrides;
        mask / dmask: the appearance mask [3,H,W] of this view and the buffer that receives dL/dmask (both contiguous
        float32 on the device), or None.
        Raises when the optimizer's tensors are no longer the ones the argument blocks point at (call rebind())."""
        from .diff_gaussian_rasterization import _C
        if self._pointers() != self._bound:
            raise RuntimeError("native step: the parameters or their Adam moments were replaced (densify, prune, "
                               "reset_opacity, load_state_dict); call rebind() first")
        a = self.args[k]
        a.view.prefix_per_tile = int(_C.PREFIX_PER_TILE)
        a.view.capacity_ctx = _C.current_capacity_context()
        if sh_degree is not None:
            a.view.D = int(sh_degree)
        if xyz_lr is not None:
            a.groups[0].lr = float(xyz_lr)
        if lrs:
            for i, n in enumerate(C_ORDER):
                if GROUP_NAME[n] in lrs:
                    a.groups[i].lr = float(lrs[GROUP_NAME[n]])
        for i, n in enumerate(C_ORDER):
            if prox is None:
                a.prox[i].u = a.prox[i].z = None
                continue
            u, z, coef = prox[GROUP_NAME[n]]
            a.prox[i].u, a.prox[i].z, a.prox[i].coef = u.data_ptr(), z.data_ptr(), float(coef)
        if mask is not None:
            c = self.cameras[k]
            for t in (mask, dmask):
                if t is None or not (t.is_contiguous() and t.dtype == torch.float32 and t.device == self.device
                                     and tuple(t.shape) == (3, int(c.height), int(c.width))):
                    raise RuntimeError("native step: mask and dmask must be contiguous float32 [3,H,W] on the device")
            a.mask, a.dmask = mask.data_ptr(), dmask.data_ptr()
        else:
            a.mask = a.dmask = None
        self.last_masked = mask is not None
        _lib.check(self.L.dg_train_step(C.byref(a), self.arena.fn, None, self.stream))
        self.last_view = k

    def sync(self) -> None:
        """Order the current stream after an overlapped f_dc / f_rest update (no-op without one)."""
        if getattr(self, "overlap", False):
            _lib.check(self.L.dg_train_sync(self.stream))
            self.arena.release_retired()

    def image(self, k: int | None = None) -> torch.Tensor:
        """The clamped render of the last step (shared buffer per image size)."""
        c = self.keep[1][self.last_view if k is None else k]
        return self.images_out[(int(c.height), int(c.width))]

    def loss(self) -> torch.Tensor:
        """(1 - ld) L1 + ld (1 - SSIM) [+ lm mean((mask - 1)^2)] + ls mean(prod(scaling)) of the last step (L1 of the
        masked render when the step had a mask: gaussian_trainer.py:392-408), a device scalar."""
        ld, ls = self.lambdas
        L1, ssim, sc = self.loss_buf[0], self.loss_buf[1], self.loss_buf[2]
        loss = (1.0 - ld) * L1 + ld * (1.0 - ssim)
        if self.last_masked:
            loss = loss + self.lambda_mask * self.loss_buf[3]
        return loss + ls * sc
