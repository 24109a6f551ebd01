"""The ADMM block trainer: one scene block per GPU rank, consensus over RCCL between local rounds.

Restates the ADMM phase of the reference's distributed trainer -- the slave's local iterations with the ADMM
penalty (conerf/trainers/slave_gaussian_trainer.py:100-207, gaussian_trainer.py:324-476) and the master's round
(master_gaussian_trainer.py:665-728: consensus, broadcast, dual update, primal/dual residuals, penalty adaptation
until stop_adapt_iter) -- without the RPC master: every rank owns its block, the consensus is one all_reduce of the
shared Gaussians (dogs_amd.admm.BlockConsensus), and the residuals and the penalty adaptation are computed
identically on every rank.

Per local iteration (`BlockTrainer.local_step`), as GaussianSplatTrainer.train_iteration after densify_end_iter:
    activations (sigmoid / exp / normalize, one launch each way)
    -> rasterizer forward + backward through the drop-in autograd function
    -> render()'s clamp + L1 (one launch each way), fused SSIM
    -> loss = (1 - lambda_dssim) L1 + lambda_dssim (1 - SSIM) + lambda_scale mean(prod(scaling, 1))  (:387-408)
    -> SparseGaussianAdam.step(visible) with the ADMM penalty sum_p 0.5 rho_p mse(x_p + u_p, z_p) (:410-411,
       slave :161-202) folded in as its gradient on the rows Adam updates (dg_adam_update_groups_prox): the penalty
       enters the optimisation only through those rows' gradients, so its value is only formed when logged
       (`penalty()`).
The xyz learning rate follows ExponentialLR (gaussian_trainer.py:32-62, 292-300) of the global iteration.

Per round (`ADMMRunner.round`): `interval` local iterations, then
    z = consensus(x)                       (master :538-555, every rank: its rows of the average)
    u += (1 + over_relaxation) (x - z)     (slave :100-121)
    primal = sum_k mse(z[idx_k], x_k); dual = rho mse(z_prev, z)   (master :396-456)
    rho adapted while iteration <= stop_adapt_iter                 (master :712-717)
The ADMM phase starts at densify_end_iter with z = the blocks' initial values and u = 0 (the reference enables the
penalty before its first broadcast, so its z is undefined until then; this is the DBACC initialisation its comment
names, slave :81-85).

`SequentialADMM` trains the same block split on one device, block after block, with the consensus done in
process: the single-GPU baseline of the north star's ">= 6x at 8 GPUs" wall-clock target.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.distributed as dist

from .admm import (PARAM_NAMES, RHO_NAMES, ADMMConfig, BlockConsensus, adapt_rho, initial_rho, residual_dicts,
                   residual_parts)

# optimizer group names of GaussianSplatTrainer.setup_optimizer (gaussian_trainer.py:205-230) for the six tensors in
# dogs_amd.admm.PARAM_NAMES order
GROUP_OF = {"xyz": "xyz", "features_dc": "f_dc", "features_rest": "f_rest", "scaling": "scaling",
            "quaternion": "quaternion", "opacity": "opacity"}


@dataclass
class TrainConfig:
    """optimizer.lr / loss blocks of config/gaussian_splatting/urban3d_admm.yaml."""
    position_init: float = 0.000016
    position_final: float = 0.00000016
    position_delay_mult: float = 0.01
    position_max_iterations: int = 30000
    feature: float = 0.0025
    opacity: float = 0.05
    scaling: float = 0.005
    quaternion: float = 0.001
    spatial_lr_scale: float = 1.0
    lambda_dssim: float = 0.2
    lambda_scale: float = 0.05
    sh_degree: int = 3
    start_iteration: int = 30000   # densify_end_iter: where the ADMM phase begins
    background: tuple = (0.0, 0.0, 0.0)
    anti_aliasing: bool = False    # texture.anti_aliasing


class ExponentialLR:
    """gaussian_trainer.py:32-62."""

    def __init__(self, lr_init, lr_final, lr_delay_steps=0, lr_delay_mult=1.0, max_steps=1000000):
        self.lr_init, self.lr_final = lr_init, lr_final
        self.lr_delay_steps, self.lr_delay_mult, self.max_steps = lr_delay_steps, lr_delay_mult, max_steps

    def __call__(self, step):
        if step < 0 or (self.lr_init == 0.0 and self.lr_final == 0.0):
            return 0.0
        if self.lr_delay_steps > 0:
            delay_rate = self.lr_delay_mult + (1 - self.lr_delay_mult) * np.sin(
                0.5 * np.pi * np.clip(step / self.lr_delay_steps, 0, 1))
        else:
            delay_rate = 1.0
        t = np.clip(step / self.max_steps, 0, 1)
        return float(delay_rate * np.exp(np.log(self.lr_init) * (1 - t) + np.log(self.lr_final) * t))


class ADMMBlockState:
    """One block's ADMM variables: z (the global values of its rows), u (duals), rho, the previous z."""

    def __init__(self, params: tuple, num_global: int, cfg: ADMMConfig, rho_gaussians: int | None = None):
        """rho_gaussians: the denominator of the initial penalties (setup_penalty_parameters, master :326-335: the
        pruned global count before the expanded-box selection); default num_global."""
        self.z = tuple(p.detach().clone() for p in params)
        self.z_prev = self.z
        self.u = tuple(torch.zeros_like(p) for p in params)
        self.rho = initial_rho(cfg, rho_gaussians or num_global)
        self.cfg = cfg

    def prox(self, params: tuple) -> dict:
        """{optimizer group name: (u, z, rho / numel)}: the penalty's gradient for dg_adam_update_groups_prox."""
        return {GROUP_OF[n]: (u, z, self.rho[r] / float(p.numel()))
                for n, r, p, u, z in zip(PARAM_NAMES, RHO_NAMES, params, self.u, self.z)}

    @torch.no_grad()
    def penalty(self, params: tuple) -> torch.Tensor:
        """sum_p 0.5 rho_p mse(x_p + u_p, z_p) (slave_gaussian_trainer.py:169-193), for logging."""
        tot = torch.zeros((), dtype=torch.float32, device=params[0].device)
        for r, x, u, z in zip(RHO_NAMES, params, self.u, self.z):
            tot = tot + 0.5 * self.rho[r] * torch.nn.functional.mse_loss(x + u, z)
        return tot

    @torch.no_grad()
    def update_duals(self, params: tuple, z_new: tuple) -> None:
        """u += (1 + alpha) (x - z) (slave_gaussian_trainer.py:100-121); z_prev <- z, z <- z_new."""
        f = 1.0 + self.cfg.over_relaxation_coeff
        for u, x, zz in zip(self.u, params, z_new):
            u.add_(f * (x.detach() - zz))
        self.z_prev, self.z = self.z, tuple(zz.reshape(p.shape).contiguous() for zz, p in zip(z_new, params))


class BlockTrainer:
    """Local iterations of one block (GaussianSplatTrainer.train_iteration + SlaveGaussianSplatTrainer's penalty).

    raw: dict of the block's six tensors in dogs_amd.admm.PARAM_NAMES order (xyz [N,3], features_dc [N,1,3],
    features_rest [N,M,3], scaling [N,3] raw log, quaternion [N,4] raw, opacity [N,1] raw logit); cameras: list of
    dogs_amd.camera.RasterCamera on the device; images: list of [3,H,W] float targets (same order)."""

    def __init__(self, raw: dict, cameras: list, images: list, num_global: int, admm: ADMMConfig,
                 cfg: TrainConfig | None = None, device: torch.device | None = None, seed: int = 0,
                 native: bool = True, rho_gaussians: int | None = None, overlap: bool = False):
        from .diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer, SparseGaussianAdam
        from .activations import activate
        from .fused_ssim import fused_ssim
        from .loss import clamp_l1, row_prod
        self.cfg = cfg or TrainConfig()
        self.device = device or raw["xyz"].device
        self.activate, self.clamp_l1, self.fused_ssim = activate, clamp_l1, fused_ssim
        self.row_prod = row_prod
        self.params = {n: raw[n].detach().to(self.device).contiguous().clone().requires_grad_(True)
                       for n in PARAM_NAMES}
        c = self.cfg
        lrs = {"xyz": c.position_init * c.spatial_lr_scale, "f_dc": c.feature, "f_rest": c.feature / 20.0,
               "opacity": c.opacity, "scaling": c.scaling, "quaternion": c.quaternion}
        self.opt = SparseGaussianAdam([{"params": [self.params[n]], "lr": lrs[GROUP_OF[n]], "name": GROUP_OF[n]}
                                       for n in PARAM_NAMES], lr=0.0, eps=1e-15)
        self.xyz_lr = ExponentialLR(c.position_init * c.spatial_lr_scale, c.position_final * c.spatial_lr_scale,
                                    lr_delay_mult=c.position_delay_mult, max_steps=c.position_max_iterations)
        bg = torch.tensor(c.background, dtype=torch.float32, device=self.device)
        self.rasts = [GaussianRasterizer(GaussianRasterizationSettings(
            cam.height, cam.width, cam.tanfovx, cam.tanfovy, bg, 1.0, cam.world_to_camera, cam.projective_matrix,
            c.sh_degree, cam.camera_center, False, False, bool(c.anti_aliasing), 0.0)) for cam in cameras]
        self.images = images
        self.rng = np.random.default_rng(seed)
        self.order: list[int] = []
        self.iteration = c.start_iteration
        self.admm = ADMMBlockState(self.param_tuple(), num_global, admm, rho_gaussians)
        self._last_loss = None
        self.cameras = cameras
        self.native = native
        if native:
            from .train_step import NativeTrainStep
            # overlap: the f_dc / f_rest update of each local step runs beside the next one's forward
            # (NativeTrainStep); ADMMRunner / SequentialADMM synchronise the device before the consensus reads the
            # parameters, and penalty() syncs
            self._nts = NativeTrainStep({n: self.params[n] for n in PARAM_NAMES}, self.opt, cameras, images,
                                        c.sh_degree, c.lambda_dssim, c.lambda_scale, bg, self.device,
                                        overlap=overlap, antialiasing=c.anti_aliasing)

    @property
    def last_loss(self):
        """The last iteration's loss without the ADMM penalty (a device scalar)."""
        if self.native and self._last_loss is None:
            self._last_loss = self._nts.loss()
        return self._last_loss

    @property
    def last_radii(self) -> torch.Tensor:
        return self._nts.radii if self.native else self._last_radii

    def param_tuple(self) -> tuple:
        return tuple(self.params[n] for n in PARAM_NAMES)

    def _next_view(self) -> int:
        # random camera order, reshuffled every epoch (gaussian_trainer.py:338-341)
        if not self.order:
            self.order = list(self.rng.permutation(len(self.rasts)))
        return int(self.order.pop())

    def local_step(self) -> None:
        """One training iteration (native: one dg_train_step call; else the autograd route), under the trainer's own
        adaptive-capacity context (GaussianSplatTrainer.train_iteration)."""
        with self._capacity():
            self._local_step()

    def _capacity(self):
        from .diff_gaussian_rasterization import _C
        if getattr(self, "capacity_ctx", None) is None:
            self.capacity_ctx = _C.new_capacity_context(owner=self)
        return _C.capacity_context(self.capacity_ctx)

    def _local_step(self) -> None:
        if not self.native:
            self._local_step_autograd()
            return
        self.iteration += 1
        lr = self.xyz_lr(self.iteration)
        for g in self.opt.param_groups:
            if g["name"] == "xyz":
                g["lr"] = lr
        self._nts.step(self._next_view(), lr, prox=self.admm.prox(self.param_tuple()))
        self._last_loss = None

    def local_step_autograd(self) -> torch.Tensor:
        """One training iteration through the drop-in autograd API (the reference's route: rasterizer, clamp/L1 and
        SSIM autograd functions, torch for the loss sum and the scale regulariser, SparseGaussianAdam with the
        penalty's proximal gradient); returns the loss without the penalty (a device scalar, no sync)."""
        with self._capacity():
            return self._local_step_autograd()

    def _local_step_autograd(self) -> torch.Tensor:
        self.sync()   # an overlapped native update of f_dc / f_rest may still be running
        self.iteration += 1
        for g in self.opt.param_groups:
            if g["name"] == "xyz":
                g["lr"] = self.xyz_lr(self.iteration)
        p = self.params
        k = self._next_view()
        gt = self.images[k]
        m2d = torch.zeros_like(p["xyz"], requires_grad=True)
        opac, scales, rots = self.activate(p["opacity"], p["scaling"], p["quaternion"])
        img, radii, _ = self.rasts[k](means3D=p["xyz"], means2D=m2d, opacities=opac, dc=p["features_dc"],
                                      shs=p["features_rest"], scales=scales, rotations=rots)
        img, l1 = self.clamp_l1(img, gt)
        ssim = self.fused_ssim(img.unsqueeze(0), gt.unsqueeze(0))
        c = self.cfg
        loss = (1.0 - c.lambda_dssim) * l1 + c.lambda_dssim * (1.0 - ssim) + c.lambda_scale * self.row_prod(scales).mean()
        loss.backward()
        self.opt.step(radii > 0, radii.shape[0], prox=self.admm.prox(self.param_tuple()))
        self.opt.zero_grad(set_to_none=True)
        self._last_radii = radii
        self._last_loss = loss.detach()
        return self._last_loss

    def sync(self) -> None:
        """Order the current stream after an overlapped update (overlap=True) before reading the block's tensors."""
        if self.native:
            self._nts.sync()

    def penalty(self) -> torch.Tensor:
        self.sync()
        return self.admm.penalty(self.param_tuple())


@dataclass
class RoundLog:
    iteration: int
    primal: dict
    dual: dict
    rho: dict
    adapted: bool
    seconds: dict = field(default_factory=dict)


def _adapt(state_rho: dict, primal: dict, dual: dict, cfg: ADMMConfig, iteration: int):
    """(master_gaussian_trainer.py:712-717) adapt only while iteration <= stop_adapt_iter."""
    if iteration <= cfg.stop_adapt_iter:
        return adapt_rho(state_rho, primal, dual, cfg), True
    return dict(state_rho), False


class ADMMRunner:
    """The per-rank ADMM loop: `interval` local iterations of this rank's block, then the consensus round over the
    process group.  local_step: a callable doing one local iteration (BlockTrainer.local_step by default; tests pass
    a torch-only stand-in)."""

    def __init__(self, params_fn, state: ADMMBlockState, consensus: BlockConsensus, local_step, cfg: ADMMConfig,
                 start_iteration: int):
        self.params_fn, self.state, self.cons, self.local_step, self.cfg = params_fn, state, consensus, local_step, cfg
        self.iteration = start_iteration
        self.logs: list[RoundLog] = []

    def round(self) -> RoundLog:
        t0 = time.perf_counter()
        for _ in range(self.cfg.consensus_interval):
            self.local_step()
        self.iteration += self.cfg.consensus_interval
        dev = self.state.z[0].device
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        params = tuple(p.detach() for p in self.params_fn())
        z = self.cons.consensus(params)
        self.state.update_duals(params, z)
        primal, dual = self.cons.residuals(params, self.state.z, self.state.z_prev, self.state.rho)
        self.state.rho, adapted = _adapt(self.state.rho, primal, dual, self.cfg, self.iteration)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        log = RoundLog(self.iteration, primal, dual, dict(self.state.rho), adapted,
                       {"local": t1 - t0, "consensus": time.perf_counter() - t1})
        self.logs.append(log)
        return log


class InProcessConsensus:
    """The consensus of several blocks held by one process (the sequential single-device baseline): the same
    shared-set average as BlockConsensus, with the all_reduce replaced by a sum over the blocks."""

    def __init__(self, global_indices: list, num_global: int, device):
        self.device = device
        self.num_global = int(num_global)
        cnt = torch.zeros(self.num_global, dtype=torch.int32, device=device)
        for g in global_indices:
            cnt.index_add_(0, g.to(device, torch.long), torch.ones(g.shape[0], dtype=torch.int32, device=device))
        self.visibility_count = cnt
        shared = cnt >= 2
        sid_of = torch.cumsum(shared.to(torch.int64), 0) - 1
        self.num_shared = int(shared.sum().item())
        self.count = cnt[shared].to(torch.float32).unsqueeze(-1) if self.num_shared else None
        self.loc, self.sid, self.owned = [], [], []
        owner = torch.full((max(self.num_shared, 1),), len(global_indices), dtype=torch.int32, device=device)
        for b, g in enumerate(global_indices):
            g = g.to(device, torch.long)
            loc = torch.nonzero(shared[g]).squeeze(-1)
            self.loc.append(loc)
            self.sid.append(sid_of[g[loc]])
            if self.num_shared:
                owner[self.sid[-1]] = torch.minimum(owner[self.sid[-1]], torch.full_like(self.sid[-1], b,
                                                                                        dtype=torch.int32))
        for b, g in enumerate(global_indices):
            own = torch.ones(g.shape[0], dtype=torch.bool, device=device)
            if self.num_shared:
                own[self.loc[b]] = owner[self.sid[b]] == b
            self.owned.append(own)
        self.owned_f = [o.to(torch.float64).unsqueeze(-1) for o in self.owned]

    def consensus(self, block_params: list) -> list:
        """[z_b for every block b] (gaussian_splat_consensus + broadcast, master :523-555)."""
        flats = [[p.detach().reshape(p.shape[0], -1) for p in ps] for ps in block_params]
        widths = [f.shape[1] for f in flats[0]]
        zs = [[f.clone() for f in fl] for fl in flats]
        if self.num_shared:
            buf = torch.zeros((self.num_shared, sum(widths)), dtype=torch.float32, device=self.device)
            for b, fl in enumerate(flats):
                buf.index_add_(0, self.sid[b], torch.cat([f[self.loc[b]] for f in fl], dim=1))
            buf.div_(self.count)           # average_gaussians (gaussian_splat_model.py:334-340)
            for b in range(len(flats)):
                rows = buf[self.sid[b]]
                o = 0
                for zi, w in zip(zs[b], widths):
                    zi[self.loc[b]] = rows[:, o:o + w]
                    o += w
        return [tuple(zi.reshape(p.shape) for zi, p in zip(z, ps)) for z, ps in zip(zs, block_params)]

    def residuals(self, block_params: list, zs: list, z_prevs: list, rho: dict):
        """As BlockConsensus.residuals, the blocks' parts summed in process (block order) instead of all_reduced."""
        part = torch.zeros(12, dtype=torch.float64, device=self.device)
        for b, (ps, z, zp) in enumerate(zip(block_params, zs, z_prevs)):
            part += residual_parts(ps, z, zp, self.owned_f[b])
        return residual_dicts(part.cpu(), block_params[0], True, self.num_global, rho)


class SequentialADMM:
    """All blocks of a split trained on one device, one after another, with the consensus in process: the
    single-GPU baseline the multi-GPU ADMM trainer is compared with (same iterations, same rounds)."""

    def __init__(self, blocks: list, states: list, params_fns: list, global_indices: list, num_global: int,
                 cfg: ADMMConfig, start_iteration: int, device):
        self.blocks, self.states, self.params_fns = blocks, states, params_fns
        self.cons = InProcessConsensus(global_indices, num_global, device)
        self.cfg = cfg
        self.iteration = start_iteration
        self.logs: list[RoundLog] = []
        self.device = device

    def round(self) -> RoundLog:
        t0 = time.perf_counter()
        for step in self.blocks:
            for _ in range(self.cfg.consensus_interval):
                step()
        self.iteration += self.cfg.consensus_interval
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        t1 = time.perf_counter()
        params = [tuple(p.detach() for p in f()) for f in self.params_fns]
        zs = self.cons.consensus(params)
        for st, ps, z in zip(self.states, params, zs):
            st.update_duals(ps, z)
        # every block holds the same rho (they start equal and adapt on the same residuals)
        rho = self.states[0].rho
        primal, dual = self.cons.residuals(params, [s.z for s in self.states], [s.z_prev for s in self.states], rho)
        new_rho, adapted = _adapt(rho, primal, dual, self.cfg, self.iteration)
        for st in self.states:
            st.rho = dict(new_rho)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        log = RoundLog(self.iteration, primal, dual, dict(new_rho), adapted,
                       {"local": t1 - t0, "consensus": time.perf_counter() - t1})
        self.logs.append(log)
        return log


# ---------------------------------------------------------------------------------------------------------------
# Synthetic block splits (the bench's ADMM workload): block k of a chain holds global ids
# [k n (1 - f), k n (1 - f) + n), so consecutive blocks share f n Gaussians.

def chain_block_indices(k: int, n: int, shared_frac: float) -> tuple[torch.Tensor, int, int]:
    stride = int(round(n * (1.0 - shared_frac)))
    return torch.arange(k * stride, k * stride + n), stride, stride


def make_block(k: int, num_blocks: int, n: int, W: int, H: int, views: int, shared_frac: float, device,
               seed: int = 1234, admm: ADMMConfig | None = None, cfg: TrainConfig | None = None, native: bool = True,
               overlap: bool = False):
    """Block k of a synthetic chain split: the BASELINE generator's scene (one global scene, seed `seed`, of
    num_global Gaussians; block k takes its rows), `views` seeded yaw cameras and random target images."""
    from .camera import make_camera, yaw_world_to_camera
    from .synthetic import make_scene
    gidx, stride, _ = chain_block_indices(k, n, shared_frac)
    num_global = stride * (num_blocks - 1) + n
    s = make_scene(n, W, H, seed=seed + k)
    # rows shared with the previous block start equal to its values (one global scene, as the reference's split)
    if k > 0 and shared_frac > 0:
        prev = make_scene(n, W, H, seed=seed + k - 1)
        m = n - stride
        for a in ("means3D", "dc", "sh", "raw_scales", "raw_rotations", "raw_opacities"):
            getattr(s, a)[:m] = getattr(prev, a)[stride:stride + m]
    raw = {"xyz": s.means3D, "features_dc": s.dc, "features_rest": s.sh, "scaling": s.raw_scales,
           "quaternion": s.raw_rotations, "opacity": s.raw_opacities}
    rng = np.random.default_rng(seed + 1000 * (k + 1))
    yaws = [0.0] + list(rng.uniform(-10.0, 10.0, max(views - 1, 0)))
    cams = [make_camera(W, H, 1600.0, 1600.0, world_to_camera=yaw_world_to_camera(math.radians(y))).to(device)
            for y in yaws]
    g = torch.Generator().manual_seed(seed + 7 + k)
    images = [torch.rand((3, H, W), generator=g).to(device) for _ in yaws]
    tr = BlockTrainer(raw, cams, images, num_global, admm or ADMMConfig(), cfg, device, seed=seed + k, native=native,
                      overlap=overlap)
    return tr, gidx, num_global


def distributed_trainer(rank: int, world: int, n: int, W: int, H: int, views: int, shared_frac: float, device,
                        admm: ADMMConfig | None = None, seed: int = 1234, group=None, overlap: bool = False):
    """This rank's block of a world-size chain split, its BlockConsensus and its ADMMRunner."""
    admm = admm or ADMMConfig()
    tr, gidx, num_global = make_block(rank, world, n, W, H, views, shared_frac, device, seed, admm, overlap=overlap)
    cons = BlockConsensus(gidx.to(device), num_global, group=group, device=device)
    run = ADMMRunner(tr.param_tuple, tr.admm, cons, tr.local_step, admm, tr.iteration)
    return tr, cons, run


def sequential_trainer(num_blocks: int, n: int, W: int, H: int, views: int, shared_frac: float, device,
                       admm: ADMMConfig | None = None, seed: int = 1234, overlap: bool = False):
    admm = admm or ADMMConfig()
    blocks, gidxs = [], []
    num_global = None
    for k in range(num_blocks):
        tr, gidx, num_global = make_block(k, num_blocks, n, W, H, views, shared_frac, device, seed, admm,
                                          overlap=overlap)
        blocks.append(tr)
        gidxs.append(gidx)
    seq = SequentialADMM([b.local_step for b in blocks], [b.admm for b in blocks], [b.param_tuple for b in blocks],
                         gidxs, num_global, admm, blocks[0].iteration, device)
    return blocks, seq


def barrier_time(fn, dev, world: int) -> float:
    """Wall time of fn() bracketed by a barrier and a device synchronisation, max over ranks."""
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt
