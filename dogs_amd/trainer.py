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

Options of the reference configs (GSTrainConfig.from_reference reads them from the YAML):
    geometry.mask / loss.lambda_mask / optimizer.lr.mask: the decoupled appearance embedding (dogs_amd.masks); the L1
        term is of the render times the mask, plus lambda_mask mean((mask - 1)^2), and the embedding has its own Adam
        (:171-183, 232-235, 392-401, 482-484).  Native iterations pass the mask to dg_train_step, which returns
        dL/dmask for the embedding's backward.
    geometry.depth_threshold: render(depth_threshold=...) (:376) -- scales the screen-space gradient the densification
        statistics read (both routes).
    texture.anti_aliasing: the rasterizer's antialiasing flag (both routes).
    appearance.use_trained_exposure: the per-image exposure and its Adam with its ExponentialLR (:158, 246-257,
        302-307, 478-480); such iterations take the autograd route (the exposure mixes the render's channels before the
        clamp, which the native step's fused loss does not model).
    geometry.coarse-to-fine: training_resolution (:309-319); downsampled iterations take the autograd route.
"""
from __future__ import annotations

import os
import random
from dataclasses import dataclass, field
from dataclasses import replace as dataclass_replace

import numpy as np
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
    mask: bool = False                  # geometry.mask: the appearance embedding
    lambda_mask: float = 0.0            # loss.lambda_mask
    mask_lr: float = 0.001              # optimizer.lr.mask
    depth_threshold: float = 0.0        # geometry.depth_threshold
    anti_aliasing: bool = False         # texture.anti_aliasing
    use_trained_exposure: bool = False  # appearance.use_trained_exposure
    exposure_lr_init: float = 0.01
    exposure_lr_final: float = 0.001
    exposure_lr_delay_steps: int = 0
    exposure_lr_delay_mult: float = 0.0
    exposure_max_iterations: int | None = None   # ${trainer.max_iterations}
    coarse_to_fine: bool = False        # geometry.coarse-to-fine

    @classmethod
    def from_reference(cls, config) -> "GSTrainConfig":
        """The loop's keys of a reference config (config/gaussian_splatting/*.yaml): a path, or the parsed dict.
        ${a.b} interpolations are resolved; geometry.spatial_lr_scale, when absent, is -1 (computed from the cameras
        by the trainer, gaussian_trainer.py:192-197)."""
        d = load_reference_config(config)
        g, lr, lo = d.get("geometry", {}), d.get("optimizer", {}).get("lr", {}), d.get("loss", {})
        pr, tx, ap = d.get("prune", {}) or {}, d.get("texture", {}), d.get("appearance", {}) or {}
        tr = d.get("trainer", {})
        kw = dict(
            max_iterations=int(tr.get("max_iterations", cls.max_iterations)),
            densify_start_iter=int(g["densify_start_iter"]), densify_end_iter=int(g["densify_end_iter"]),
            densification_interval=int(g["densification_interval"]),
            opacity_reset_interval=int(g["opacity_reset_interval"]),
            densify_grad_threshold=float(g["densify_grad_threshold"]), percent_dense=float(g["percent_dense"]),
            prune_iterations=tuple(int(i) for i in (pr.get("iterations") or [])),
            prune_v_pow=float(pr.get("v_pow", cls.prune_v_pow)),
            prune_decay=float(pr.get("prune_decay", cls.prune_decay)),
            prune_percent=float(pr.get("prune_percent", cls.prune_percent)),
            position_init=float(lr["position_init"]), position_final=float(lr["position_final"]),
            position_delay_mult=float(lr["position_delay_mult"]),
            position_max_iterations=int(lr["position_max_iterations"]),
            feature=float(lr["feature"]), opacity=float(lr["opacity"]), scaling=float(lr["scaling"]),
            quaternion=float(lr["quaternion"]), mask_lr=float(lr.get("mask", cls.mask_lr)),
            exposure_lr_init=float(lr.get("exposure_lr_init", cls.exposure_lr_init)),
            exposure_lr_final=float(lr.get("exposure_lr_final", cls.exposure_lr_final)),
            exposure_lr_delay_steps=int(lr.get("exposure_lr_delay_steps", cls.exposure_lr_delay_steps)),
            exposure_lr_delay_mult=float(lr.get("exposure_lr_delay_mult", cls.exposure_lr_delay_mult)),
            exposure_max_iterations=int(lr["exposure_max_iterations"]) if "exposure_max_iterations" in lr else None,
            lambda_dssim=float(lo["lambda_dssim"]), lambda_scale=float(lo["lambda_scale"]),
            lambda_mask=float(lo.get("lambda_mask", 0.0) or 0.0),
            max_sh_degree=int(tx.get("max_sh_degree", cls.max_sh_degree)),
            anti_aliasing=bool(tx.get("anti_aliasing", False)),
            spatial_lr_scale=float(g.get("spatial_lr_scale", -1)),
            white_background=bool(d.get("dataset", {}).get("apply_mask", False)),
            mask=bool(g.get("mask", False)), depth_threshold=float(g.get("depth_threshold", 0) or 0.0),
            use_trained_exposure=bool(ap.get("use_trained_exposure", False)),
            coarse_to_fine=bool(g.get("coarse-to-fine", False)),
        )
        return cls(**kw)


def _resolve(node, root):
    if isinstance(node, dict):
        return {k: _resolve(v, root) for k, v in node.items()}
    if isinstance(node, list):
        return [_resolve(v, root) for v in node]
    if isinstance(node, str) and node.startswith("${") and node.endswith("}") and node.count("${") == 1:
        cur = root
        for part in node[2:-1].split("."):
            cur = cur[part]
        return _resolve(cur, root)
    return node


def load_reference_config(config) -> dict:
    """A reference YAML config (path or already-parsed dict) with its whole-value ${a.b} interpolations resolved
    (what OmegaConf returns for the keys the trainers read)."""
    import yaml
    if isinstance(config, (str, os.PathLike)):
        with open(config, "r", encoding="utf-8") as f:
            config = yaml.safe_load(f)
    return _resolve(config, config)


def nerf_plus_plus_norm(cameras: list) -> float:
    """compute_nerf_plus_plus_norm (conerf/datasets/utils.py:352-369) as the reference evaluates it: each camera
    centre becomes a [1, 3] row and np.hstack joins them into [1, 3n], so the "centre" is the mean of all 3n
    coordinates and the diagonal the largest |coordinate - that mean|; radius = 1.1 x diagonal."""
    rows = [c.camera_center.detach().reshape(1, 3).cpu().numpy() for c in cameras]
    centers = np.hstack(rows)
    center = np.mean(centers, axis=1, keepdims=True)
    diagonal = np.max(np.linalg.norm(centers - center, axis=0, keepdims=True))
    return float(diagonal * 1.1)


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
    on the device; images: [3,H,W] float targets (same order); bounding_box: the scene's [6] box or None;
    appear_embedding: an existing dogs_amd.masks.AppearanceEmbedding (the reference constructor's argument; with
    cfg.mask and none given, one is built over len(cameras) views).  A camera's image_index selects its embedding row
    and exposure (its position in `cameras` when it has none)."""

    def __init__(self, model: GaussianSplatModel, cameras: list, images: list, cfg: GSTrainConfig | None = None,
                 device=None, seed: int = 0, native: bool = True, bounding_box=None, normal=torch.normal,
                 overlap: bool = True, appear_embedding=None):
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
        # geometry.spatial_lr_scale < 0: the cameras' radius (setup_training_params, gaussian_trainer.py:192-197)
        s = c.spatial_lr_scale if c.spatial_lr_scale >= 0 else nerf_plus_plus_norm(cameras)
        self.spatial_lr_scale = s
        lrs = {"xyz": c.position_init * s, "f_dc": c.feature, "f_rest": c.feature / 20.0, "opacity": c.opacity,
               "scaling": c.scaling, "quaternion": c.quaternion}
        self.optimizer = SparseGaussianAdam([{"params": [p], "lr": lrs[n], "name": n}
                                             for n, p in model.params().items()], lr=0.0, eps=1e-15)
        self.xyz_scheduler = ExponentialLR(c.position_init * s, c.position_final * s,
                                           lr_delay_mult=c.position_delay_mult,
                                           max_steps=c.position_max_iterations or c.max_iterations)
        # the appearance embedding and its Adam (:171-183, 232-235)
        self.mask = appear_embedding
        if self.mask is None and c.mask:
            from .masks import AppearanceEmbedding
            self.mask = AppearanceEmbedding(len(cameras))
        self.mask_optimizer = None
        self._masked = None
        if self.mask is not None:
            from .masks import MaskedStep
            self.mask = self.mask.to(self.device)
            # torch's fused Adam on the GPU: one launch per step instead of ~8 foreach kernels (~100 us per masked
            # iteration); the same optimizer in both routes and in every ADMM rank
            self.mask_optimizer = torch.optim.Adam(self.mask.parameters(), lr=c.mask_lr,
                                                   fused=self.device.type == "cuda")
            self._masked = MaskedStep(self.mask, self.mask_optimizer)
        # the trained exposure and its Adam + schedule (:246-257); the model holds one [3,4] per training image
        self.exposure_optimizer = self.exposure_scheduler = None
        if c.use_trained_exposure:
            if model.get_exposure.numel() == 0:
                model.init_exposure([self._image_index(k) for k in range(len(cameras))])
            self.exposure_optimizer = torch.optim.Adam([model.get_exposure])
            self.exposure_scheduler = ExponentialLR(c.exposure_lr_init, c.exposure_lr_final,
                                                    lr_delay_steps=c.exposure_lr_delay_steps,
                                                    lr_delay_mult=c.exposure_lr_delay_mult,
                                                    max_steps=c.exposure_max_iterations or c.max_iterations)
        self._nts = None
        self._nts_stats = None
        self.last_loss = None
        self._scaled_views: dict = {}

    # ---- helpers
    def _image_index(self, k: int) -> int:
        idx = getattr(self.cameras[k], "image_index", -1)
        return int(idx) if idx is not None and int(idx) >= 0 else k

    def _stats_on(self) -> bool:
        return self.iteration < self.cfg.densify_end_iter

    def _stats(self) -> dict:
        m = self.model
        return {"max_radii2D": m.max_radii2D, "grad_accum": m.xyz_gradient_accum, "denom": m.denom}

    def _params(self) -> dict:
        m = self.model
        return {"xyz": m._xyz, "features_dc": m._features_dc, "features_rest": m._features_rest,
                "opacity": m._opacity, "scaling": m._scaling, "quaternion": m._quaternion}

    def _native_step(self):
        from .train_step import C_ORDER, NativeTrainStep
        want_stats = self._stats_on()
        if self._nts is None or self._nts_stats != want_stats:
            m, c = self.model, self.cfg
            params = self._params()
            assert tuple(params) == C_ORDER
            if self._nts is None:
                self._nts = NativeTrainStep(params, self.optimizer, self.cameras, self.images, m.active_sh_degree,
                                            c.lambda_dssim, c.lambda_scale, self.bg, self.device,
                                            stats=self._stats() if want_stats else None, overlap=self.overlap,
                                            lambda_mask=c.lambda_mask, depth_threshold=c.depth_threshold,
                                            antialiasing=c.anti_aliasing)
            else:
                self._nts.rebind(params, self._stats() if want_stats else None)
            self._nts_stats = want_stats
        return self._nts

    def _rebind(self):
        if self._nts is not None:
            self._nts.rebind(self._params(), self._stats() if self._stats_on() else None)
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

    def training_resolution(self) -> int:
        """gaussian_trainer.py:309-319: 4, 2, then 1 over the first min(20000, densify_end_iter) iterations."""
        if not self.cfg.coarse_to_fine:
            return 1
        n_interval = 3
        threshold = min(20000, self.cfg.densify_end_iter) // n_interval
        return 2 ** max(n_interval - self.iteration // threshold - 1, 0)

    def _view_at(self, k: int, resolution: int):
        """(camera, target) of view k at a training resolution (Camera.downsample: the image through Resize)."""
        if resolution == 1:
            return self.cameras[k], self.images[k]
        key = (k, resolution)
        v = self._scaled_views.get(key)
        if v is None:
            from .masks import downsample_image
            v = self._scaled_views[key] = (self.cameras[k].downsample(resolution),
                                           downsample_image(self.images[k], resolution).contiguous())
        return v

    def update_learning_rate(self) -> float:
        lr = self.xyz_scheduler(self.iteration)
        for g in self.optimizer.param_groups:
            if g["name"] == "xyz":
                g["lr"] = lr
        if self.exposure_scheduler is not None:   # _update_exposure_params_lr (:302-307)
            for g in self.exposure_optimizer.param_groups:
                g["lr"] = self.exposure_scheduler(self.iteration)
        return lr

    # ---- one iteration
    def train_iteration(self) -> IterationLog:
        # the trainer's own adaptive-capacity context: its views' phase split, instance numbering and gradient-sum
        # rounding do not depend on anything else this process rendered (dg_raster_args.capacity_ctx)
        from .diff_gaussian_rasterization import _C
        if getattr(self, "capacity_ctx", None) is None:
            self.capacity_ctx = _C.new_capacity_context(owner=self)
        with _C.capacity_context(self.capacity_ctx):
            return self._train_iteration()

    def _train_iteration(self) -> IterationLog:
        c = self.cfg
        self.iteration += 1
        lr = self.update_learning_rate()
        if self.iteration % c.sh_increase_interval == 0:
            self.model.increase_SH_degree()
        k = self._next_view()
        ev = self._events()
        res = self.training_resolution()
        if self.native and not ev and res == 1 and self.exposure_optimizer is None:
            nts = self._native_step()
            mask = dmask = None
            if self._masked is not None:
                mask, dmask = self._masked.forward(k, self.images[k], self._image_index(k))
            nts.step(k, lr, sh_degree=self.model.active_sh_degree, mask=mask, dmask=dmask)
            if self._masked is not None:
                self._masked.backward_and_step(dmask)
            self.last_loss = None
            log = IterationLog(self.iteration, "native", self.model.num_gaussians)
        else:
            self.sync()
            self._autograd_iteration(k, ev, res)
            log = IterationLog(self.iteration, "autograd", self.model.num_gaussians, ev)
        self.logs.append(log)
        return log

    def _autograd_iteration(self, k: int, ev: list, resolution: int = 1) -> None:
        from .densify import densify_and_prune
        from .fused_ssim import fused_ssim
        from .loss import row_prod
        from .prune import calculate_v_imp_score, prune_list
        from .render import render
        c, m = self.cfg, self.model
        cam, gt = self._view_at(k, resolution)
        if self.exposure_optimizer is not None and getattr(cam, "image_index", -1) < 0:
            cam = dataclass_replace(cam, image_index=self._image_index(k))
        out = render(m, cam, _Pipe, self.bg, anti_aliasing=c.anti_aliasing, separate_sh=True,
                     use_trained_exposure=c.use_trained_exposure, depth_threshold=c.depth_threshold,
                     device=self.device)
        colors, ssp, vis, radii = out["rendered_image"], out["screen_space_points"], out["visibility_filter"], \
            out["radii"]
        loss_ssim = fused_ssim(colors.unsqueeze(0), gt.unsqueeze(0))
        if self.mask is not None:   # :392-401 -- the mask from the full-resolution target, 32x downsampled
            from .masks import MASK_DOWNSAMPLE
            small = self._masked.small_target(k, self.images[k]) if resolution == 1 else None
            if small is None:
                from .masks import downsample_image
                small = downsample_image(self.images[k], MASK_DOWNSAMPLE)
            mask = self.mask(small, self._image_index(k), tuple(gt.shape[1:]))
            l1 = F.l1_loss(colors * mask, gt)
            loss = (1.0 - c.lambda_dssim) * l1 + c.lambda_dssim * (1.0 - loss_ssim) + \
                c.lambda_mask * torch.mean((mask - 1) ** 2.)
        else:
            l1 = F.l1_loss(colors, gt)
            loss = (1.0 - c.lambda_dssim) * l1 + c.lambda_dssim * (1.0 - loss_ssim)
        loss = loss + c.lambda_scale * row_prod(out["scaling"]).mean()
        loss.backward()
        self.last_loss = loss.detach()
        replaced = False
        with torch.no_grad():
            if self.iteration < c.densify_end_iter:
                m.add_densification_stats(ssp, vis, radii)
                if "densify" in ev:
                    size_threshold = 20 if self.iteration > c.opacity_reset_interval else None
                    densify_and_prune(m, c.densify_grad_threshold, c.min_opacity, self.spatial_lr_scale,
                                      size_threshold, self.optimizer, self.bounding_box, normal=self.normal)
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
        if self.exposure_optimizer is not None:    # :478-480
            self.exposure_optimizer.step()
            self.exposure_optimizer.zero_grad(set_to_none=True)
        if self.mask_optimizer is not None:        # :482-484
            self.mask_optimizer.step()
            self.mask_optimizer.zero_grad(set_to_none=True)
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
