"""The ADMM phase entry: from per-block models trained independently up to densify_end_iter to the consensus phase's
block split (MasterGaussianSplatTrainer.fuse_local_gaussians, conerf/trainers/master_gaussian_trainer.py:557-618),
without the RPC master.

Reference order (rank 0's master, once, at the first round with iteration >= densify_end_iter):
    1. fuse_block_gaussians (:37-100): every block's model clipped to its ORIGINAL point box in the oriented-bbox frame
       (points_in_bbox2D of x, y), then concatenated in block order;
    2. prune_gaussians_after_merge (:103-121): prune_list over every block's cameras (LightGaussian count renders of
       the fused model) -> calculate_v_imp_score -> prune_gaussians(0.4 * prune_percent);
    3. num_gaussians = the pruned count, the denominator of the initial penalties (setup_penalty_parameters, :326-335);
    4. select_gaussians_in_each_block (:124-172): the Gaussians inside no EXPANDED box are dropped, then each block
       takes the Gaussians inside its expanded box (overlaps belong to several blocks), visibility_count = bincount;
    5. new block trainers from the sub-models, penalties set, duals set up, ADMM enabled.

Here every rank runs the entry for its own block ("one block per GPU"):
    * each rank clips its block to its original box first (the reference clips per block too, so the rows that cross
      the wire are only the ones the fused model keeps), then the clipped rows are all-gathered (variable row
      counts: one all_gather of the sizes, one of the rows padded to the largest block into one flat buffer), so
      every rank fuses the same global model -- clipping, concatenation, the box tests and the prune compaction are
      deterministic, so the ranks agree bit for bit without further exchange.  Memory: every rank holds the fused
      model, 236 B per Gaussian (config 5, 8 blocks x ~5e6 clipped: ~9.4 GB of a rank's 288 GB of HBM), as the
      reference's master does once; the gather's peak is the padded buffer plus the fused copy (2x), freed before the
      count renders.  The count renders need the whole fused model on every rank that renders (any Gaussian can
      occlude any camera's pixels), which is why it is gathered rather than sharded;
    * the count renders are split across ranks: rank r renders its own block's cameras only, keeping each camera's
      score vector (cameras x 4 B per fused Gaussian);
    * the importance is then summed in the reference's exact order: prune_gaussians_after_merge concatenates the
      blocks' camera lists and prune_list pops from the end, so the float32 sum is one left fold over block B-1's
      cameras (last first), then block B-2's, ..., then block 0's.  The fold runs as a chain over the ranks
      (rank B-1 folds its scores and sends the [N] partial to rank B-2, which folds its own onto it, ...; the adds are
      cheap next to the renders, which all ranks did in parallel), and rank 0 broadcasts the total.  The result is
      bit-identical to prune_list over the concatenated list, so the percentile threshold of v_imp_prune keeps and
      drops the same Gaussians as the reference;
    * the expanded-box split, visibility_count and the rank's sub-model follow locally.
`enter_admm_phase_sequential` runs the same entry in one process with prune_list over the concatenated camera list
(the reference's own order; the tests compare the two bit for bit).

The device work goes through `PhaseKernels` (HIP: dg_rasterize_count, dg_points_in_boxes2d, dg_prune_select +
dg_densify_gather); the CPU tests substitute restatements of the same three operations to check the distributed
plumbing with gloo.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

from .admm import PARAM_NAMES
from .gaussian_model import GaussianSplatModel, percentile_mask


@dataclass
class PhaseConfig:
    """prune block of the config (urban3d_admm.yaml / mill19: prune.prune_percent, prune.v_pow)."""
    prune_percent: float = 0.5
    v_pow: float = 0.1
    merge_prune_factor: float = 0.4    # prune_gaussians_after_merge: 0.4 * prune_percent (:119)


class PhaseKernels:
    """The phase entry's device operations (HIP)."""

    def camera_importance(self, model: GaussianSplatModel, camera, bg: torch.Tensor) -> torch.Tensor:
        """count_render's important_score of one camera, float32 [N]."""
        from .prune import count_render
        cam = camera.to(model.get_xyz.device) if hasattr(camera, "to") else camera
        return count_render(model, cam, None, bg)["important_score"]

    def importance(self, model: GaussianSplatModel, cameras: list, bg: torch.Tensor) -> torch.Tensor:
        """prune_list's important_score summed over `cameras` (last camera first, one float32 left fold), [N]."""
        acc = torch.zeros(model.num_gaussians, dtype=torch.float32, device=model.get_xyz.device)
        for cam in reversed(list(cameras)):
            acc += self.camera_importance(model, cam, bg)
        return acc

    def members(self, xy: torch.Tensor, boxes: list, transform) -> list:
        """[ascending int64 indices of the points inside each closed box (in the OBB frame)]."""
        from .blocksplit import points_in_boxes2d
        out = []
        for i in range(0, len(boxes), 64):
            out += points_in_boxes2d(xy, [np.asarray(b, dtype=np.float64).reshape(2, 3)[:, :2]
                                          for b in boxes[i:i + 64]], transform, device=xy.device)["members"]
        return out

    def prune(self, model: GaussianSplatModel, mask: torch.Tensor) -> None:
        model.prune_points(mask, None)


def _flat(model: GaussianSplatModel) -> torch.Tensor:
    """[N, 59] rows (xyz, f_dc, f_rest, scaling, quaternion, opacity: get_all_properties order)."""
    ts = model.get_all_properties()
    n = ts[0].shape[0]
    return torch.cat([t.detach().reshape(n, -1).float() for t in ts], dim=1).contiguous()


def _split_rows(rows: torch.Tensor, like: GaussianSplatModel) -> tuple:
    shapes = [tuple(t.shape[1:]) for t in like.get_all_properties()]
    out, o = [], 0
    n = rows.shape[0]
    for s in shapes:
        w = int(np.prod(s)) if s else 1
        out.append(rows[:, o:o + w].reshape((n,) + s).contiguous())
        o += w
    return tuple(out)


def _gather_device(group) -> torch.device | None:
    """gloo's all_gather takes host tensors; RCCL device tensors."""
    return torch.device("cpu") if dist.get_backend(group) == "gloo" else None


def all_gather_rows(rows: torch.Tensor, group=None) -> torch.Tensor:
    """Every rank's [n_r, D] rows (n_r may differ) concatenated in rank order, [sum n_r, D]: one all_gather of the
    sizes, one of the rows padded to max n_r into one flat buffer (the peak is that buffer plus the result; gloo on host
    tensors, RCCL on device tensors)."""
    world = dist.get_world_size(group)
    host = _gather_device(group)
    dev = rows.device
    src = rows.to(host) if host is not None else rows
    n = torch.tensor([rows.shape[0]], dtype=torch.int64, device=src.device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    sizes = [int(x.item()) for x in ns]
    nmax = max(sizes) if sizes else 0
    d = rows.shape[1]
    pad = src if src.shape[0] == nmax else torch.cat(
        [src, torch.zeros((nmax - src.shape[0], d), dtype=src.dtype, device=src.device)], 0)
    flat = torch.empty((world * nmax, d), dtype=rows.dtype, device=src.device)
    dist.all_gather_into_tensor(flat, pad.contiguous(), group=group)
    del pad, src
    if not all(s == nmax for s in sizes):
        flat = torch.cat([flat[r * nmax:r * nmax + s] for r, s in enumerate(sizes)], 0)
    return flat.to(dev)


def clip_block(model: GaussianSplatModel, box, world_to_obb_transform, kernels: PhaseKernels) -> torch.Tensor:
    """fuse_block_gaussians' per-block step (master_gaussian_trainer.py:37-100): the [n, 59] rows of `model` inside
    its ORIGINAL point box (OBB frame); every row when `box` is None."""
    rows = _flat(model)
    if box is None:
        return rows
    keep = kernels.members(model.get_xyz.detach()[:, :2], [box], world_to_obb_transform)[0]
    return rows[keep.to(rows.device)]


def _fused_model(rows: torch.Tensor, like: GaussianSplatModel) -> GaussianSplatModel:
    fused = GaussianSplatModel(like.max_sh_degree, like.percent_dense, like.get_xyz.device)
    fused.init_from_external_properties(*_split_rows(rows, like), optimizable=False)
    # the master's model is created with active_sh_degree = max_sh_degree (master_gaussian_trainer.py:216-220), and
    # the blocks' sub-models inherit it (get_sub_gaussians, gaussian_splat_model.py:290-306)
    fused.active_sh_degree = like.max_sh_degree
    return fused


def fuse_blocks(block_models: list, ori_point_bboxes, world_to_obb_transform, kernels: PhaseKernels):
    """fuse_block_gaussians (master_gaussian_trainer.py:37-100) without its PLY side outputs: each block clipped to
    its original box (OBB frame), concatenated in block order.  Returns the fused (non-optimisable) model."""
    parts = [clip_block(m, None if ori_point_bboxes is None else ori_point_bboxes[b], world_to_obb_transform, kernels)
             for b, m in enumerate(block_models)]
    return _fused_model(torch.cat(parts, 0), block_models[0])


def ordered_importance(fused: GaussianSplatModel, camera_blocks: list, kernels: PhaseKernels, bg: torch.Tensor,
                       group=None, score_budget_bytes: int = 1 << 30) -> torch.Tensor:
    """prune_list's importance over the concatenation of every block's cameras, bit for bit, with each rank rendering
    only its own block's cameras: the per-camera scores are folded down a chain of ranks in the reference's order
    (block B-1's last camera first ... block 0's first camera last), and broadcast from rank 0.

    While a rank waits for the partial sum of the ranks after it, it renders its first cameras ahead and keeps their
    scores -- at most `score_budget_bytes` of them (4 B per fused Gaussian per camera: 200 cameras of a 4e7-Gaussian
    fused model would be 32 GB) -- then folds them in order and renders the rest straight into the sum.  The last
    rank starts the chain from zeros and buffers nothing."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = fused.get_xyz.device
    n = fused.num_gaussians
    cams = list(reversed(list(camera_blocks[rank])))
    ahead = 0 if rank == world - 1 else min(len(cams), int(score_budget_bytes) // max(4 * n, 1))
    own = [kernels.camera_importance(fused, cam, bg).float() for cam in cams[:ahead]]
    host = _gather_device(group)
    wire = host if host is not None else dev
    acc = torch.zeros(n, dtype=torch.float32, device=dev)
    if rank < world - 1:
        buf = torch.empty(n, dtype=torch.float32, device=wire)
        dist.recv(buf, src=dist.get_global_rank(group, rank + 1) if group is not None else rank + 1, group=group)
        acc = buf.to(dev)
    for sc in own:
        acc += sc
    del own
    for cam in cams[ahead:]:
        acc += kernels.camera_importance(fused, cam, bg).float()
    if rank > 0:
        dist.send(acc.to(wire), dst=dist.get_global_rank(group, rank - 1) if group is not None else rank - 1,
                  group=group)
    out = acc.to(wire)
    dist.broadcast(out, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    return out.to(dev)


def v_imp_prune(model: GaussianSplatModel, imp: torch.Tensor, cfg: PhaseConfig, kernels: PhaseKernels) -> None:
    """calculate_v_imp_score + prune_gaussians(0.4 * prune_percent) (master :117-119, prune.py:14-32,
    gaussian_splat_model.py:420-432)."""
    from .prune import calculate_v_imp_score
    v = calculate_v_imp_score(model, imp, cfg.v_pow)
    kernels.prune(model, percentile_mask(v, cfg.merge_prune_factor * cfg.prune_percent))


def select_gaussians_in_each_block(bboxes: list, model: GaussianSplatModel, world_to_obb_transform,
                                   kernels: PhaseKernels, blocks=None):
    """master_gaussian_trainer.py:124-172: drop the Gaussians inside no expanded box, then (visibility_count [N],
    global_indices [per block, ascending int64], sub-models of `blocks` (default: every block))."""
    xy = model.get_xyz.detach()[:, :2]
    mem = kernels.members(xy, bboxes, world_to_obb_transform)
    n = model.num_gaussians
    cnt = torch.zeros(n, dtype=torch.int64, device=xy.device)
    for m in mem:
        cnt.index_add_(0, m.to(xy.device), torch.ones_like(m, device=xy.device))
    valid = torch.nonzero(cnt).squeeze(-1)
    if valid.numel() != n:
        model.extract_sub_gaussians(valid)
        xy = model.get_xyz.detach()[:, :2]
        mem = kernels.members(xy, bboxes, world_to_obb_transform)
    n = model.num_gaussians
    vis = torch.zeros(n, dtype=torch.int64, device=xy.device)
    for m in mem:
        vis.index_add_(0, m.to(xy.device), torch.ones_like(m, device=xy.device))
    assert bool((vis != 0).all()), "visibility count has zero elements!"
    want = range(len(bboxes)) if blocks is None else blocks
    subs = {b: model.get_sub_gaussians(mem[b]) for b in want}
    return vis, [m.to(torch.int64) for m in mem], subs


@dataclass
class PhaseEntry:
    """What a rank needs to start the ADMM phase: its block's optimisable sub-model, its global indices, the
    visibility count of the global set, the global count and the penalty denominator (the pruned count)."""
    model: GaussianSplatModel
    global_indices: torch.Tensor
    visibility_count: torch.Tensor
    num_global: int
    rho_gaussians: int
    fused: GaussianSplatModel
    timings: dict | None = None  # per stage seconds, with DOGS_ENTRY_TIMING=1 (device-synchronised stage by stage)

    def raw(self) -> dict:
        """The sub-model as BlockTrainer's raw dict (dogs_amd.admm.PARAM_NAMES)."""
        m = self.model
        return dict(zip(PARAM_NAMES, (m._xyz, m._features_dc, m._features_rest, m._scaling, m._quaternion,
                                      m._opacity)))


def enter_admm_phase(block_model: GaussianSplatModel, camera_blocks: list, ori_point_bboxes: list,
                     exp_point_bboxes: list, world_to_obb_transform=None, cfg: PhaseConfig | None = None,
                     kernels: PhaseKernels | None = None, group=None, bg: torch.Tensor | None = None) -> PhaseEntry:
    """This rank's part of fuse_local_gaussians (master_gaussian_trainer.py:557-618) over the process group: rank r
    holds block r's model (trained up to densify_end_iter) and camera_blocks[b] lists block b's cameras (every rank
    knows the split, as every reference worker reads the block folders)."""
    cfg = cfg or PhaseConfig()
    kernels = kernels or PhaseKernels()
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if len(camera_blocks) != world:
        raise RuntimeError(f"{len(camera_blocks)} camera blocks for {world} ranks (one block per rank)")
    dev = block_model.get_xyz.device
    bg = torch.zeros(3, dtype=torch.float32, device=dev) if bg is None else bg
    timings = {} if os.environ.get("DOGS_ENTRY_TIMING") == "1" else None
    t = [time.perf_counter()]

    def stage(name):
        if timings is not None:
            torch.cuda.synchronize(dev)
            t.append(time.perf_counter())
            timings[name] = t[-1] - t[-2]
    # 1. every rank clips its own block to its original box (the reference's per-block fuse step), the clipped rows
    #    are all-gathered in block order and every rank builds the same fused model from them
    clipped = clip_block(block_model, None if ori_point_bboxes is None else ori_point_bboxes[rank],
                         world_to_obb_transform, kernels)
    stage("clip")
    rows = all_gather_rows(clipped, group)
    del clipped
    stage("gather")
    fused = _fused_model(rows, block_model)
    del rows
    stage("fuse")
    # 2. importance: this rank renders its cameras only, summed in the reference's order down the rank chain
    imp = ordered_importance(fused, camera_blocks, kernels, bg, group)
    stage("importance")
    v_imp_prune(fused, imp, cfg, kernels)
    rho_gaussians = fused.num_gaussians
    stage("prune")
    # 4. the expanded-box split
    vis, gidx, subs = select_gaussians_in_each_block(exp_point_bboxes, fused, world_to_obb_transform, kernels,
                                                     blocks=[rank])
    stage("split")
    return PhaseEntry(subs[rank], gidx[rank], vis, int(vis.shape[0]), rho_gaussians, fused, timings)


def enter_admm_phase_sequential(block_models: list, camera_blocks: list, ori_point_bboxes: list,
                                exp_point_bboxes: list, world_to_obb_transform=None, cfg: PhaseConfig | None = None,
                                kernels: PhaseKernels | None = None, bg: torch.Tensor | None = None) -> list:
    """The same entry for every block in one process (the single-GPU baseline, and the restatement the distributed
    entry is tested against): [PhaseEntry per block]."""
    cfg = cfg or PhaseConfig()
    kernels = kernels or PhaseKernels()
    dev = block_models[0].get_xyz.device
    bg = torch.zeros(3, dtype=torch.float32, device=dev) if bg is None else bg
    fused = fuse_blocks(block_models, ori_point_bboxes, world_to_obb_transform, kernels)
    # prune_gaussians_after_merge (:103-121): prune_list over the blocks' concatenated camera lists
    imp = kernels.importance(fused, [c for cams in camera_blocks for c in cams], bg).float().reshape(-1)
    v_imp_prune(fused, imp, cfg, kernels)
    rho_gaussians = fused.num_gaussians
    vis, gidx, subs = select_gaussians_in_each_block(exp_point_bboxes, fused, world_to_obb_transform, kernels)
    return [PhaseEntry(subs[b], gidx[b], vis, int(vis.shape[0]), rho_gaussians, fused)
            for b in range(len(exp_point_bboxes))]
