"""ADMM block consensus over RCCL (one scene block per GPU, no master process).

Replaces the RPC gather/average/scatter of the reference master trainer
(conerf/trainers/master_gaussian_trainer.py:459-555, gaussian_splat_model.py:316-340) and the per-block
ADMM state of the slave (slave_gaussian_trainer.py:100-202) with collectives between block ranks:

* Gaussians that live in exactly one block have z = x_k and a dual that never moves, so only the
  *shared* set (visibility_count >= 2) is exchanged.  Each rank packs its shared rows of the six raw
  parameter tensors (59 floats per Gaussian) into one [N_shared, 59] buffer (zeros where it holds no
  copy).  The sum is an all-reduce built from two collectives so that its order is the reference
  master's: all_to_all hands rank r every rank's copy of row slice r, rank r adds them in block order
  onto zeros and divides by the count (reinitialize + plus_gaussians per block + average_gaussians,
  gaussian_splat_model.py:316-340, master_gaussian_trainer.py:538-555), all_gather returns the
  slices.  Same bytes on the wire as a ring all_reduce ((W-1)/W of the buffer each way, twice), and the
  result is bit-identical to the reference's arithmetic and to the sequential baseline for every
  count, not only where the sum has two terms.
* Primal/dual residuals are per-rank partial sums, gathered (12 scalars per rank) and added in rank
  order; every shared Gaussian is owned (counted once) by the lowest rank that holds it.
* Penalty adaptation (master_gaussian_trainer.py:337-377) is deterministic given the residuals, so
  every rank applies it locally -- no broadcast.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist
import torch.nn.functional as F

PARAM_NAMES = ("xyz", "features_dc", "features_rest", "scaling", "quaternion", "opacity")
RHO_NAMES = ("xyz", "fdc", "fr", "s", "q", "o")


@dataclass
class ADMMConfig:
    """trainer.admm block of the reference configs (config/gaussian_splatting/urban3d_admm.yaml:42-55)."""
    consensus_interval: int = 200
    alpha_xyz: float = 1e5
    alpha_fdc: float = 1e4
    alpha_fr: float = 1e5
    alpha_s: float = 1e4
    alpha_q: float = 1e5
    alpha_o: float = 1e4
    stop_adapt_iter: int = 32000
    mu: float = 10.0
    tau_inc: float = 2.0
    tau_dec: float = 2.0
    over_relaxation_coeff: float = 0.5


def _flat(t: torch.Tensor) -> torch.Tensor:
    return t.reshape(t.shape[0], -1)


class BlockConsensus:
    """Consensus state of one block rank.

    global_indices: this rank's global Gaussian ids (the reference's global_indices[k]).
    visibility_count: [N_global] number of blocks holding each Gaussian (torch.bincount of all blocks'
    indices, master_gaussian_trainer.py:163-168); when None it is built with one all_reduce.
    """

    def __init__(self, global_indices: torch.Tensor, num_global: int, visibility_count: torch.Tensor | None = None,
                 group=None, device: torch.device | None = None):
        self.group = group
        self.device = device or global_indices.device
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        gidx = global_indices.to(self.device, torch.long)
        self.gidx = gidx
        self.num_global = int(num_global)
        if visibility_count is None:
            cnt = torch.zeros(self.num_global, dtype=torch.int32, device=self.device)
            cnt.index_add_(0, gidx, torch.ones_like(gidx, dtype=torch.int32))
            if self.world > 1:
                dist.all_reduce(cnt, op=dist.ReduceOp.SUM, group=group)
            visibility_count = cnt
        vc = visibility_count.to(self.device)
        self.visibility_count = vc
        shared = vc >= 2
        sid_of = torch.cumsum(shared.to(torch.int64), 0) - 1
        self.num_shared = int(shared.sum().item())
        loc_mask = shared[gidx]
        self.loc = torch.nonzero(loc_mask).squeeze(-1)                    # local rows of shared Gaussians
        self.sid = sid_of[gidx[self.loc]]                                # their compact shared ids
        # float32 count per shared row: `x /= count` with an int64 count promotes to a float32 division
        self.count = vc[shared].to(torch.float32).unsqueeze(-1) if self.num_shared else None
        # owner of each shared Gaussian = lowest rank holding it (counts it in the dual residual)
        owner = torch.full((max(self.num_shared, 1),), self.world, dtype=torch.int32, device=self.device)
        if self.num_shared:
            owner[self.sid] = self.rank
            if self.world > 1:
                dist.all_reduce(owner, op=dist.ReduceOp.MIN, group=group)
        own = torch.ones(gidx.shape[0], dtype=torch.bool, device=self.device)
        if self.num_shared:
            own[self.loc] = owner[self.sid] == self.rank
        self.owned = own
        self._owned_f = None
        self.widths: tuple[int, ...] | None = None

    # ---------------------------------------------------------------------------------------------
    def consensus(self, params: tuple[torch.Tensor, ...]) -> tuple[torch.Tensor, ...]:
        """z_k = (sum over blocks of x at the same global id) / count, for this block's rows.
        Restates gaussian_splat_consensus + broadcast_global_gaussian_splat (master_gaussian_trainer.py:523-555)."""
        flats = [_flat(p.detach()) for p in params]
        widths = tuple(f.shape[1] for f in flats)
        self.widths = widths
        z = [f.clone() for f in flats]
        if self.num_shared:
            D = sum(widths)
            buf = torch.zeros((self.num_shared, D), dtype=torch.float32, device=self.device)
            buf[self.sid] = torch.cat([f[self.loc] for f in flats], dim=1)
            if self.world > 1:
                buf = ordered_sum_average(buf, self.count, self.world, self.rank, self.group)
            else:
                buf = torch.zeros_like(buf).add_(buf).div_(self.count)
            rows = buf[self.sid]
            o = 0
            for zi, w in zip(z, widths):
                zi[self.loc] = rows[:, o:o + w]
                o += w
        return tuple(zi.reshape(p.shape) for zi, p in zip(z, params))

    @torch.no_grad()
    def update_duals(self, duals: list[torch.Tensor], params: tuple[torch.Tensor, ...],
                     z: tuple[torch.Tensor, ...], over_relaxation_coeff: float) -> None:
        """u += (1 + alpha) (x - z)  (slave_gaussian_trainer.py:100-121)."""
        f = 1.0 + over_relaxation_coeff
        for u, x, zz in zip(duals, params, z):
            u.add_(f * (x.detach() - zz))

    @torch.no_grad()
    def residuals(self, params: tuple[torch.Tensor, ...], z: tuple[torch.Tensor, ...],
                  z_prev: tuple[torch.Tensor, ...] | None, rho: dict[str, float]) -> tuple[dict, dict]:
        """Primal: sum over blocks of MSE(z[idx_k], x_k) (master_gaussian_trainer.py:396-433).
        Dual: rho * MSE(z_prev, z) over the global set (:435-456), each Gaussian counted once."""
        if self._owned_f is None or self._owned_f.shape[0] != self.owned.shape[0]:
            self._owned_f = self.owned.to(torch.float64).unsqueeze(-1)
        part = residual_parts(params, z, z_prev, self._owned_f)
        if self.world > 1:
            parts = torch.empty((self.world * part.shape[0],), dtype=part.dtype, device=part.device)
            dist.all_gather_into_tensor(parts, part, group=self.group)
            parts = parts.view(self.world, -1)
            part = torch.zeros_like(part)
            for k in range(self.world):          # rank order, as the sequential baseline adds its blocks
                part += parts[k]
        return residual_dicts(part.cpu(), params, z_prev is not None, self.num_global, rho)


@torch.no_grad()
def ordered_sum_average(buf: torch.Tensor, count: torch.Tensor, world: int, rank: int, group=None) -> torch.Tensor:
    """(sum over ranks of buf, added in rank order onto zeros) / count, on every rank.

    buf is [S, D] (this rank's copies, zeros elsewhere), count [S, 1] float32.  Row slice r of the padded
    buffer is reduced by rank r: all_to_all delivers the W copies of the slice, they are added in rank
    order (0 + x_0 + x_1 + ...: the reference master's reinitialize + plus_gaussians loop), divided by the
    count, and all_gather_into_tensor reassembles the [S, D] result."""
    S, D = buf.shape
    chunk = -(-S // world)
    pad = chunk * world
    if pad != S:
        buf = torch.cat([buf, buf.new_zeros((pad - S, D))])
        count = torch.cat([count, count.new_ones((pad - S, 1))])
    recv = torch.empty_like(buf)
    dist.all_to_all_single(recv, buf, group=group)
    recv = recv.view(world, chunk, D)
    acc = torch.zeros((chunk, D), dtype=buf.dtype, device=buf.device)
    for k in range(world):
        acc += recv[k]
    acc.div_(count[rank * chunk:(rank + 1) * chunk])
    out = torch.empty_like(buf)
    dist.all_gather_into_tensor(out, acc, group=group)
    return out[:S]


@torch.no_grad()
def residual_parts(params, z, z_prev, owned_f: torch.Tensor) -> torch.Tensor:
    """[12] float64 on the device, no host sync: MSE(z, x) per tensor, then the owned rows' sum of (z_prev - z)^2."""
    part = torch.zeros(12, dtype=torch.float64, device=owned_f.device)
    for i, (x, zz) in enumerate(zip(params, z)):
        part[i] = F.mse_loss(zz.float(), x.detach().float()).double()
        if z_prev is not None:
            d = (_flat(z_prev[i]) - _flat(zz)).double() * owned_f
            part[6 + i] = (d * d).sum()
    return part


def residual_dicts(part: torch.Tensor, params, have_prev: bool, num_global: int, rho: dict):
    """(primal, dual) dicts from the summed parts (one host copy)."""
    v = part.tolist()
    primal = {n: float(v[i]) for i, n in enumerate(RHO_NAMES)}
    dual = {}
    for i, n in enumerate(RHO_NAMES):
        per = int(_flat(params[i]).shape[1])
        dual[n] = rho[n] * float(v[6 + i]) / float(num_global * per) if have_prev else 0.0
    return primal, dual


def initial_rho(cfg: ADMMConfig, num_gaussians: int) -> dict[str, float]:
    """setup_penalty_parameters (master_gaussian_trainer.py:326-335)."""
    s = 1.0 / num_gaussians
    return {"xyz": s * cfg.alpha_xyz, "fdc": s * cfg.alpha_fdc, "fr": s * cfg.alpha_fr, "s": s * cfg.alpha_s,
            "q": s * cfg.alpha_q, "o": s * cfg.alpha_o}


def adapt_rho(rho: dict[str, float], primal: dict, dual: dict, cfg: ADMMConfig) -> dict[str, float]:
    """adapt_penalty_parameters (master_gaussian_trainer.py:337-377)."""
    out = dict(rho)
    for n in RHO_NAMES:
        if primal[n] > cfg.mu * dual[n]:
            out[n] = rho[n] * cfg.tau_inc
        elif dual[n] > cfg.mu * primal[n]:
            out[n] = rho[n] / cfg.tau_dec
    return out


def admm_penalty(params: tuple[torch.Tensor, ...], duals: list[torch.Tensor], z: tuple[torch.Tensor, ...],
                 rho: dict[str, float]) -> torch.Tensor:
    """sum_p 0.5 rho_p MSE(x_p + u_p, z_p)  (slave_gaussian_trainer.py:161-202)."""
    tot = None
    for n, x, u, zz in zip(RHO_NAMES, params, duals, z):
        t = 0.5 * rho[n] * F.mse_loss(x + u, zz)
        tot = t if tot is None else tot + t
    return tot
