"""The single-GPU 3DGS training loop: GaussianSplatTrainer.train_iteration (conerf/trainers/gaussian_trainer.py:324-513)
inside ImplicitReconTrainer.train (conerf/trainers/implicit_recon_trainer.py:296-353), BASELINE config 2's loop.

Per iteration, in the reference's order:
    iteration += 1; xyz lr = ExponentialLR(iteration) (:287-300); every 1000 iterations increase_SH_degree (:328-329)
    camera: a random permutation of the training views per epoch (:336-341)
    render -> loss = (1 - l_dssim) L1 + l_dssim (1 - fused SSIM) + l_scale mean(prod(scaling)) -> backward
    while iteration < densify_end_iter: max_radii2D / densification statistics (:429-438); every
        densification_interval after densify_start_iter: densify_and_prune (:440-451); every opacity_reset_interval:
        reset_opacity (:453-455)
    at each prune.iterations entry: LightGaussian prune_list -> calculate_v_imp_score -> prune_gaussians_with_opt
        (:457-470)
    SparseGaussianAdam.step(radii > 0, N) (:472-476) -- a group whose tensor was just replaced has no gradient and is
        skipped, exactly as in the reference (densify / prune iterations update nothing, a reset skips the opacity).

Routes.  Ordinary iterations run as one dg_train_step call (dogs_amd.train_step: activations, forward, clamp + L1,
SSIM, backward, scale regulariser, Adam and the densification statistics, the kernels of the autograd route);
iterations that densify, reset or prune run the autograd route (dogs_amd.render + SparseGaussianAdam), because the
reference replaces the tensors between the backward and the optimizer step.  After such an iteration the native step
is rebound to the new tensors (NativeTrainStep.rebind; its pointer check refuses a stale binding).
`native=False` runs every iteration through the autograd route (the drop-in API as the reference's trainer calls it).
"""
from __future__ import annotations

import random
from dataclasses import dataclass, field

import torch
import torch.nn.functional as F

from .admm_trainer import ExponentialLR
from .gaussian_model import GaussianSplatModel


@dataclass
class GSTrainConfig:
    """The keys of config/gaussian_splatting/mipnerf360.yaml the loop consumes (trainer, prune, optimizer.lr,
    geometry, texture, loss blocks)."""
    max_iterations: int = 30000
    densify_start_iter: int = 500
    densify_end_iter: int = 15000
    densification_interval: int = 100
    opacity_reset_interval: int = 3000
    densify_grad_threshold: float = 0.0002
    percent_dense: float = 0.01
    min_opacity: float = 0.005          # gaussian_trainer.py:446
    prune_iterations: tuple = ()        # prune.iterations ([16000, 24000] in the commented default)
    prune_v_pow: float = 0.1
    prune_decay: float = 0.6
    prune_percent: float = 0.5
    position_init: float = 0.00016
    position_final: float = 0.0000016
    position_delay_mult: float = 0.01
    position_max_iterations: int | None = None   # ${trainer.max_iterations}
    feature: float = 0.0025
    opacity: float = 0.025
    scaling: float = 0.005
    quaternion: float = 0.001
    lambda_dssim: float = 0.2
    lambda_scale: float = 0.01
    max_sh_degree: int = 3
    spatial_lr_scale: float = 1.0
    white_background: bool = False      # use_white_bkgd (dataset.apply_mask): reset at densify_start_iter too
    background: tuple = (0.0, 0.0, 0.0)
    sh_increase_interval: int = 1000    # gaussian_trainer.py:328


@dataclass
class IterationLog:
    iteration: int
    route: str
    num_gaussians: int
    events: list = field(default_factory=list)


class _Pipe:
    debug = False
    compute_cov3D_python = False
    convert_SHs_python = False


class GaussianSplatTrainer:
    """model: dogs_amd.gaussian_model.GaussianSplatModel (optimisable tensors on the device); cameras: RasterCameras
    on the device; images: [3,H,W] float targets (same order); bounding_box: the scene's [6] box or None."""

    def __init__(self, model: GaussianSplatModel, cameras: list, images: list, cfg: GSTrainConfig | None = None,
                 device=None, seed: int = 0, native: bool = True, bounding_box=None, normal=torch.normal,
                 overlap: bool = True):
        from .diff_gaussian_rasterization import SparseGaussianAdam
        self.cfg = c = cfg or GSTrainConfig()
        # overlap: native steps return with their f_dc / f_rest update still running on a side stream (NativeTrainStep);
        # the autograd-route iterations and train()'s end call sync() first -- call it before reading the model
        # after train_iteration() yourself
        self.overlap = overlap
        self.model = model
        self.device = torch.device(device) if device is not None else model.get_xyz.device
        self.cameras, self.images = cameras, images
        self.bg = torch.tensor(c.background, dtype=torch.float32, device=self.device)
        self.iteration = 0
        self.rng = random.Random(seed)
        self.order: list[int] = []
        self.native = native
        self.bounding_box = bounding_box
        self.normal = normal
        self.logs: list[IterationLog] = []
        s = c.spatial_lr_scale
        lrs = {"xyz": c.position_init * s, "f_dc": c.feature, "f_rest": c.feature / 20.0, "opacity": c.opacity,
               "scaling": c.scaling, "quaternion": c.quaternion}
        self.optimizer = SparseGaussianAdam([{"params": [p], "lr": lrs[n], "name": n}
                                             for n, p in model.params().items()], lr=0.0, eps=1e-15)
        self.xyz_scheduler = ExponentialLR(c.position_init * s, c.position_final * s,
                                           lr_delay_mult=c.position_delay_mult,
                                           max_steps=c.position_max_iterations or c.max_iterations)
        self._nts = None
        self._nts_stats = None
        self.last_loss = None

    # ---- helpers
    def _stats_on(self) -> bool:
        return self.iteration < self.cfg.densify_end_iter

    def _stats(self) -> dict:
        m = self.model
        return {"max_radii2D": m.max_radii2D, "grad_accum": m.xyz_gradient_accum, "denom": m.denom}

    def _native_step(self):
        from .train_step import C_ORDER, NativeTrainStep
        want_stats = self._stats_on()
        if self._nts is None or self._nts_stats != want_stats:
            m = self.model
            params = {"xyz": m._xyz, "features_dc": m._features_dc, "features_rest": m._features_rest,
                      "opacity": m._opacity, "scaling": m._scaling, "quaternion": m._quaternion}
            assert tuple(params) == C_ORDER
            if self._nts is None:
                self._nts = NativeTrainStep(params, self.optimizer, self.cameras, self.images, m.active_sh_degree,
                                            self.cfg.lambda_dssim, self.cfg.lambda_scale, self.bg, self.device,
                                            stats=self._stats() if want_stats else None, overlap=self.overlap)
            else:
                self._nts.rebind(params, self._stats() if want_stats else None)
            self._nts_stats = want_stats
        return self._nts

    def _rebind(self):
        if self._nts is not None:
            m = self.model
            self._nts.rebind({"xyz": m._xyz, "features_dc": m._features_dc, "features_rest": m._features_rest,
                              "opacity": m._opacity, "scaling": m._scaling, "quaternion": m._quaternion},
                             self._stats() if self._stats_on() else None)
            self._nts_stats = self._stats_on()

    def _next_view(self) -> int:
        if not self.order:
            self.order = list(range(len(self.cameras)))
            self.rng.shuffle(self.order)
        return self.order.pop()

    def _events(self) -> list:
        """What this iteration does after its backward (gaussian_trainer.py:429-470)."""
        c, it = self.cfg, self.iteration
        ev = []
        if it < c.densify_end_iter:
            if it > c.densify_start_iter and it % c.densification_interval == 0:
                ev.append("densify")
            if it % c.opacity_reset_interval == 0 or (c.white_background and it == c.densify_start_iter):
                ev.append("reset_opacity")
        if it in list(c.prune_iterations):
            ev.append("prune")
        return ev

    def update_learning_rate(self) -> float:
        lr = self.xyz_scheduler(self.iteration)
        for g in self.optimizer.param_groups:
            if g["name"] == "xyz":
                g["lr"] = lr
        return lr

    # ---- one iteration
    def train_iteration(self) -> IterationLog:
        c = self.cfg
        self.iteration += 1
        lr = self.update_learning_rate()
        if self.iteration % c.sh_increase_interval == 0:
            self.model.increase_SH_degree()
        k = self._next_view()
        ev = self._events()
        if self.native and not ev:
            nts = self._native_step()
            nts.step(k, lr, sh_degree=self.model.active_sh_degree)
            self.last_loss = None
            log = IterationLog(self.iteration, "native", self.model.num_gaussians)
        else:
            self.sync()
            self._autograd_iteration(k, ev)
            log = IterationLog(self.iteration, "autograd", self.model.num_gaussians, ev)
        self.logs.append(log)
        return log

    def _autograd_iteration(self, k: int, ev: list) -> None:
        from .densify import densify_and_prune
        from .fused_ssim import fused_ssim
        from .prune import calculate_v_imp_score, prune_list
        from .render import render
        c, m = self.cfg, self.model
        cam, gt = self.cameras[k], self.images[k]
        out = render(m, cam, _Pipe, self.bg, separate_sh=True, device=self.device)
        colors, ssp, vis, radii = out["rendered_image"], out["screen_space_points"], out["visibility_filter"], \
            out["radii"]
        loss_ssim = fused_ssim(colors.unsqueeze(0), gt.unsqueeze(0))
        l1 = F.l1_loss(colors, gt)
        loss = (1.0 - c.lambda_dssim) * l1 + c.lambda_dssim * (1.0 - loss_ssim)
        loss = loss + c.lambda_scale * out["scaling"].prod(dim=1).mean()
        loss.backward()
        self.last_loss = loss.detach()
        replaced = False
        with torch.no_grad():
            if self.iteration < c.densify_end_iter:
                m.add_densification_stats(ssp, vis, radii)
                if "densify" in ev:
                    size_threshold = 20 if self.iteration > c.opacity_reset_interval else None
                    densify_and_prune(m, c.densify_grad_threshold, c.min_opacity, c.spatial_lr_scale, size_threshold,
                                      self.optimizer, self.bounding_box, normal=self.normal)
                    replaced = True
                if "reset_opacity" in ev:
                    m.reset_opacity(self.optimizer)
                    replaced = True
            if "prune" in ev:
                _, imp = prune_list(m, self.cameras, _Pipe, self.bg)
                v = calculate_v_imp_score(m, imp, c.prune_v_pow)
                i = list(c.prune_iterations).index(self.iteration)
                m.prune_gaussians_with_opt((c.prune_decay ** i) * c.prune_percent, v, self.optimizer)
                replaced = True
        self.optimizer.step(radii > 0, radii.shape[0])
        self.optimizer.zero_grad(set_to_none=True)
        if replaced:
            self._rebind()

    def loss(self) -> torch.Tensor:
        """The last iteration's loss (a device scalar)."""
        if self.last_loss is None and self._nts is not None:
            return self._nts.loss()
        return self.last_loss

    def sync(self) -> None:
        """Order the current stream after the native step's overlapped SH update (overlap=True), so that the model's
        tensors and Adam moments can be read or replaced; train() ends with it."""
        if self._nts is not None:
            self._nts.sync()

    def train(self, iterations: int | None = None) -> None:
        """ImplicitReconTrainer.train's loop (checkpoints, validation and logging are not on the path)."""
        end = self.cfg.max_iterations if iterations is None else self.iteration + iterations
        while self.iteration < end:
            self.train_iteration()
        self.sync()
