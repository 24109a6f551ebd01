"""The distributed ADMM run, end to end, one block per rank (`torchrun --nproc-per-node B ... -m dogs_amd.admm_run`).

Restates MasterGaussianSplatTrainer.train / train_iteration (conerf/trainers/master_gaussian_trainer.py:620-728) and
the workers it drives (slave_gaussian_trainer.py:204-207, gaussian_trainer.py:324-513), launched as
scripts/train/train_admm_master.sh:34-42 launches them, without the RPC master:

  1. pre-phase: every rank trains its block with GaussianSplatTrainer (densification, opacity resets, LightGaussian
     prunes, the appearance mask, depth_threshold -- the block config's loop) in consensus_interval chunks, until the
     iteration reaches densify_end_iter (the master returns from train_iteration while iteration < densify_end_iter,
     :686-688);
  2. the phase entry (fuse_local_gaussians, :557-618 -> dogs_amd.admm_phase.enter_admm_phase): the blocks fused and
     clipped to their original boxes, pruned once by importance over all cameras, re-split by the expanded boxes;
  3. the ADMM phase: a fresh block trainer per rank (the reference re-creates its workers from the sub-models: new
     SparseGaussianAdam, no appearance mask -- `sub_masks` is None at :560/609), then rounds of consensus_interval
     local steps + consensus over the process group until max_iterations (:665-728).
The master's consensus right after the entry (the same train_iteration, :690-692 then :694-717) averages blocks whose
shared rows are all copies of the same fused row, so z = x, u = 0 and both residuals are 0: it is the initial state
ADMMBlockState starts from, and no exchange is spent on it.

`run_sequential` runs the same split on one device, block after block (the single-GPU baseline of the north star's
">= 6x at 8 GPUs"; the tests hold the distributed run to it).
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.distributed as dist

from .admm import ADMMConfig, BlockConsensus
from .admm_phase import PhaseConfig, PhaseEntry, enter_admm_phase, enter_admm_phase_sequential
from .admm_trainer import ADMMRunner, BlockTrainer, SequentialADMM, TrainConfig
from .gaussian_model import GaussianSplatModel
from .trainer import GaussianSplatTrainer, GSTrainConfig, load_reference_config


@dataclass
class ADMMRunConfig:
    gs: GSTrainConfig = field(default_factory=GSTrainConfig)
    admm: ADMMConfig = field(default_factory=ADMMConfig)
    native: bool = True
    overlap: bool = True

    @classmethod
    def from_reference(cls, config) -> "ADMMRunConfig":
        """trainer / geometry / prune / optimizer / loss blocks and trainer.admm of a reference config
        (config/gaussian_splatting/urban3d_admm.yaml)."""
        d = load_reference_config(config)
        a = d.get("trainer", {}).get("admm", {}) or {}
        kw = {}
        for k, typ in (("consensus_interval", int), ("alpha_xyz", float), ("alpha_fdc", float), ("alpha_fr", float),
                       ("alpha_s", float), ("alpha_q", float), ("alpha_o", float), ("stop_adapt_iter", int),
                       ("mu", float), ("tau_inc", float), ("tau_dec", float), ("over_relaxation_coeff", float)):
            if k in a:
                kw[k] = typ(float(a[k])) if typ is int else typ(a[k])
        return cls(gs=GSTrainConfig.from_reference(d), admm=ADMMConfig(**kw))


@dataclass
class BlockScene:
    """What rank b reads (the block folders of load_colmap's split): every block's cameras -- the phase entry renders
    each block's cameras on that block's rank, and the split must be known everywhere -- this block's training
    targets and initial point cloud (points3D_{b}.ply), the original / expanded point boxes and the world-to-OBB
    transform (bounding_boxes*.txt, world_to_obb_transform.npy)."""
    camera_blocks: list              # [block][RasterCamera] on the device
    images: list                     # [3,H,W] float targets of camera_blocks[block]
    points: np.ndarray               # [n,3]
    colors: np.ndarray               # [n,3] in [0, 1]
    ori_boxes: list
    exp_boxes: list
    transform: np.ndarray | None
    block: int = 0
    bounding_box: torch.Tensor | None = None


@dataclass
class RankRun:
    pre: GaussianSplatTrainer
    entry: PhaseEntry
    block: BlockTrainer
    consensus: BlockConsensus
    runner: ADMMRunner
    seconds: dict


def _normal(device, seed: int):
    g = torch.Generator(device=device).manual_seed(seed)
    return lambda mean, std: torch.normal(mean, std, generator=g)


def _mask_net(cfg: GSTrainConfig, n_views: int, seed: int):
    """The block's AppearanceEmbedding, initialised from a per-block seed (the same on any rank or process)."""
    if not cfg.mask:
        return None
    from .masks import AppearanceEmbedding
    with torch.random.fork_rng(devices=[]):
        torch.manual_seed(seed)
        return AppearanceEmbedding(n_views)


def pre_phase_trainer(cfg: ADMMRunConfig, scene: BlockScene, device, seed: int = 0) -> GaussianSplatTrainer:
    """The block's worker before the ADMM phase (init_gaussians from the block's points, build_networks, setup)."""
    gs = cfg.gs
    b = scene.block
    cams = scene.camera_blocks[b]
    model = GaussianSplatModel(gs.max_sh_degree, gs.percent_dense, device)
    idxs = [c.image_index if getattr(c, "image_index", -1) >= 0 else k for k, c in enumerate(cams)]
    model.init_from_colmap_pcd(scene.points, scene.colors, image_idxs=idxs if gs.use_trained_exposure else None)
    return GaussianSplatTrainer(model, cams, scene.images, gs, device=device, seed=seed + 101 * b, native=cfg.native,
                                bounding_box=scene.bounding_box, normal=_normal(device, seed + 7 * b + 1),
                                overlap=cfg.overlap, appear_embedding=_mask_net(gs, len(cams), seed + 13 * b))


def pre_phase_iterations(cfg: ADMMRunConfig) -> int:
    """Iterations before the entry: consensus_interval chunks until >= densify_end_iter (0 when it is <= 0)."""
    d, k = cfg.gs.densify_end_iter, cfg.admm.consensus_interval
    return 0 if d <= 0 else int(math.ceil(d / k)) * k


def block_train_config(cfg: ADMMRunConfig, pre: GaussianSplatTrainer, start_iteration: int,
                       sh_degree: int) -> TrainConfig:
    """The re-created worker's setup (setup_training_params / setup_optimizer): the same optimizer.lr and loss keys,
    the same spatial_lr_scale (same cameras), continuing at the master's iteration (update_iteration)."""
    gs = cfg.gs
    return TrainConfig(position_init=gs.position_init, position_final=gs.position_final,
                       position_delay_mult=gs.position_delay_mult,
                       position_max_iterations=gs.position_max_iterations or gs.max_iterations,
                       feature=gs.feature, opacity=gs.opacity, scaling=gs.scaling, quaternion=gs.quaternion,
                       spatial_lr_scale=pre.spatial_lr_scale, lambda_dssim=gs.lambda_dssim,
                       lambda_scale=gs.lambda_scale, sh_degree=sh_degree, start_iteration=start_iteration,
                       background=gs.background, anti_aliasing=gs.anti_aliasing)


def run(cfg: ADMMRunConfig, scene: BlockScene, group=None, device=None, seed: int = 0, kernels=None,
        max_rounds: int | None = None) -> RankRun:
    """This rank's whole run (scene.block = its rank in `group`).  max_rounds caps the ADMM rounds (None: until
    max_iterations)."""
    rank = dist.get_rank(group)
    if scene.block != rank:
        raise RuntimeError(f"rank {rank} was given block {scene.block}: one block per rank, in rank order")
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    secs = {}
    t0 = time.perf_counter()
    pre = pre_phase_trainer(cfg, scene, dev, seed)
    n_pre = pre_phase_iterations(cfg)
    while pre.iteration < n_pre:            # train_every_x_interval chunks (the master's RPC rounds)
        pre.train(cfg.admm.consensus_interval)
    pre.sync()
    # the entry starts with a collective: without this barrier its time would include the wait for the slowest rank's
    # pre-phase (the per-phase times are maxima over ranks; the wall clock is the same either way)
    if dist.get_world_size(group) > 1:
        dist.barrier(group=group)
    secs["pre_phase"] = time.perf_counter() - t0
    t1 = time.perf_counter()
    pc = PhaseConfig(prune_percent=cfg.gs.prune_percent, v_pow=cfg.gs.prune_v_pow)
    entry = enter_admm_phase(pre.model, scene.camera_blocks, scene.ori_boxes, scene.exp_boxes, scene.transform, pc,
                             kernels, group, pre.bg)
    secs["entry"] = time.perf_counter() - t1
    cams = scene.camera_blocks[rank]
    tcfg = block_train_config(cfg, pre, n_pre, entry.model.active_sh_degree)
    blk = BlockTrainer(entry.raw(), cams, scene.images, entry.num_global, cfg.admm, tcfg, dev, seed=seed + 31 * rank,
                       native=cfg.native, rho_gaussians=entry.rho_gaussians, overlap=cfg.overlap)
    cons = BlockConsensus(entry.global_indices, entry.num_global, visibility_count=entry.visibility_count,
                          group=group, device=dev)
    runner = ADMMRunner(blk.param_tuple, blk.admm, cons, blk.local_step, cfg.admm, n_pre)
    t2 = time.perf_counter()
    rounds = 0
    while runner.iteration < cfg.gs.max_iterations and (max_rounds is None or rounds < max_rounds):
        runner.round()
        rounds += 1
    blk.sync()
    secs["admm"] = time.perf_counter() - t2
    return RankRun(pre, entry, blk, cons, runner, secs)


@dataclass
class SequentialRun:
    pres: list
    entries: list
    blocks: list
    seq: SequentialADMM
    seconds: dict


def run_sequential(cfg: ADMMRunConfig, scenes: list, device, seed: int = 0, kernels=None,
                   max_rounds: int | None = None) -> SequentialRun:
    """The same run for every block on one device, one block after another (scenes[b].block == b)."""
    dev = torch.device(device)
    secs = {}
    t0 = time.perf_counter()
    n_pre = pre_phase_iterations(cfg)
    pres = []
    for sc in scenes:
        pre = pre_phase_trainer(cfg, sc, dev, seed)
        while pre.iteration < n_pre:
            pre.train(cfg.admm.consensus_interval)
        pre.sync()
        pres.append(pre)
    secs["pre_phase"] = time.perf_counter() - t0
    t1 = time.perf_counter()
    sc0 = scenes[0]
    pc = PhaseConfig(prune_percent=cfg.gs.prune_percent, v_pow=cfg.gs.prune_v_pow)
    entries = enter_admm_phase_sequential([p.model for p in pres], sc0.camera_blocks, sc0.ori_boxes, sc0.exp_boxes,
                                          sc0.transform, pc, kernels, pres[0].bg)
    secs["entry"] = time.perf_counter() - t1
    blocks = []
    for b, (sc, e) in enumerate(zip(scenes, entries)):
        tcfg = block_train_config(cfg, pres[b], n_pre, e.model.active_sh_degree)
        blocks.append(BlockTrainer(e.raw(), sc.camera_blocks[b], sc.images, e.num_global, cfg.admm, tcfg, dev,
                                   seed=seed + 31 * b, native=cfg.native, rho_gaussians=e.rho_gaussians,
                                   overlap=cfg.overlap))
    seq = SequentialADMM([t.local_step for t in blocks], [t.admm for t in blocks], [t.param_tuple for t in blocks],
                         [e.global_indices for e in entries], entries[0].num_global, cfg.admm, n_pre, dev)
    t2 = time.perf_counter()
    rounds = 0
    while seq.iteration < cfg.gs.max_iterations and (max_rounds is None or rounds < max_rounds):
        seq.round()
        rounds += 1
    for t in blocks:
        t.sync()
    secs["admm"] = time.perf_counter() - t2
    return SequentialRun(pres, entries, blocks, seq, secs)


# ---------------------------------------------------------------------------------------------------------------
# A synthetic aerial scene split by the Grid2D path (tests, the bench's ADMM leg): points on a ground slab, nadir
# cameras on a regular grid above it, the split through cluster_image_in_grid / cluster_points_in_grid.

def aerial_views(n_points: int, cams_x: int, cams_y: int, W: int, H: int, extent=4.0, height: float = 6.0,
                 seed: int = 0) -> dict:
    """{'points' [n,3] f64, 'colors' [n,3] u8, 'camtoworlds' [C,4,4] f64, 'fx', 'W', 'H'} of a ground slab
    [-ex, ex] x [-ey, ey] x [-0.3, 0.3] (extent = e or (ex, ey)) seen by cams_x x cams_y nadir cameras at `height`
    (70 degrees of horizontal field of view)."""
    ex, ey = (float(extent), float(extent)) if np.isscalar(extent) else (float(extent[0]), float(extent[1]))
    rng = np.random.default_rng(seed)
    pts = np.stack([rng.uniform(-ex, ex, n_points), rng.uniform(-ey, ey, n_points),
                    rng.uniform(-0.3, 0.3, n_points)], 1)
    cols = rng.integers(0, 256, (n_points, 3)).astype(np.uint8)
    c2w = []
    for j in range(cams_y):
        for i in range(cams_x):
            cx = -ex + (i + 0.5) * 2 * ex / cams_x
            cy = -ey + (j + 0.5) * 2 * ey / cams_y
            m = np.eye(4)
            m[:3, :3] = np.diag([1.0, -1.0, -1.0])       # camera z = world -z (looking down)
            m[:3, 3] = (cx, cy, height)
            c2w.append(m)
    fx = 0.5 * W / math.tan(math.radians(35.0))
    return {"points": pts, "colors": cols, "camtoworlds": np.stack(c2w), "fx": fx, "W": W, "H": H}


def split_scene(views: dict, mx: int, my: int, save_dir: str, device, bbox_scale=(1.4, 1.4, 1.4),
                image_seed: int = 0) -> list:
    """[BlockScene per block] of aerial_views through the Grid2D split (load_colmap.py:98-177) and block export
    (:459-487).  Targets: seeded smooth random images (the synthetic scene has no photographs)."""
    from .blockio import export_blocks
    from .blocksplit import cluster_image_in_grid, cluster_points_in_grid, points_in_bbox2D
    c2w = views["camtoworlds"]
    n_img = c2w.shape[0]
    names = [f"img_{i:04d}" for i in range(n_img)]
    v = {"image_names": names, "camtoworlds": c2w,
         "intrinsics": np.stack([np.array([[views["fx"], 0, views["W"] / 2], [0, views["fx"], views["H"] / 2],
                                           [0, 0, 1.0]])] * n_img),
         "sizes": np.array([[views["W"], views["H"]]] * n_img, dtype=np.int64)}
    nb = mx * my
    ids, _, _, _ = cluster_image_in_grid(c2w, save_dir, list(range(n_img)), list(bbox_scale),
                                         {i: i + 1 for i in range(n_img)}, num_blocks=nb, mx=mx, my=my)
    bb, ebb, T = cluster_points_in_grid(views["points"], views["colors"], save_dir, list(bbox_scale), num_blocks=nb,
                                        mx=mx, my=my)
    ds = export_blocks(save_dir, v, ids)
    dev = torch.device(device)
    cams = [[c.raster_camera(dev) for c in d.cameras] for d in ds]
    g = torch.Generator().manual_seed(image_seed)
    scenes = []
    imgs_all = {}
    for b in range(nb):
        imgs = []
        for c in ds[b].cameras:
            if c.image_path not in imgs_all:      # one target per image, shared by the blocks that hold it
                lo = torch.rand((1, 3, 8, 8), generator=g)
                imgs_all[c.image_path] = torch.nn.functional.interpolate(
                    lo, size=(c.height, c.width), mode="bilinear", align_corners=False)[0].contiguous()
            imgs.append(imgs_all[c.image_path].to(dev))
        sel = points_in_bbox2D(views["points"][:, :2], ebb[b].reshape(2, 3), T)
        scenes.append(BlockScene(cams, imgs, views["points"][sel], views["colors"][sel] / 255.0,
                                 [x.reshape(-1) for x in bb], [x.reshape(-1) for x in ebb], T, b))
    return scenes


def main(argv=None) -> None:
    """torchrun entry over the synthetic aerial split (one block per rank; RCCL on GPUs, gloo with --gloo):
    python -m torch.distributed.run --nproc-per-node B -m dogs_amd.admm_run --mx 2 --my 2 [--config yaml]."""
    import argparse
    import json
    import os
    import tempfile
    p = argparse.ArgumentParser()
    p.add_argument("--config", default=None, help="a reference YAML (urban3d_admm.yaml); default: the built-in keys")
    p.add_argument("--mx", type=int, default=2)
    p.add_argument("--my", type=int, default=1)
    p.add_argument("--points", type=int, default=20000)
    p.add_argument("--width", type=int, default=320)
    p.add_argument("--height", type=int, default=240)
    # schedule overrides: applied only when given (with --config the YAML's schedule and prunes stand otherwise);
    # without --config the defaults are a short synthetic run (densify to 200, 600 iterations, rounds of 100)
    p.add_argument("--densify-end", type=int, default=None)
    p.add_argument("--max-iterations", type=int, default=None)
    p.add_argument("--interval", type=int, default=None)
    p.add_argument("--gloo", action="store_true")
    a = p.parse_args(argv)
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    if world != a.mx * a.my:
        raise SystemExit(f"world size {world} != mx * my = {a.mx * a.my} (one block per rank)")
    local = int(os.environ.get("LOCAL_RANK", 0))
    dev = torch.device("cuda", 0 if a.gloo else local)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo" if a.gloo else "nccl", rank=rank, world_size=world)
    cfg = ADMMRunConfig.from_reference(a.config) if a.config else None
    if cfg is None:
        cfg = ADMMRunConfig()
        a.densify_end = 200 if a.densify_end is None else a.densify_end
        a.max_iterations = 600 if a.max_iterations is None else a.max_iterations
        a.interval = 100 if a.interval is None else a.interval
        cfg.gs.prune_iterations = ()
    if a.densify_end is not None:
        cfg.gs.densify_end_iter = a.densify_end
        cfg.gs.densify_start_iter = min(cfg.gs.densify_start_iter, a.densify_end // 2)
        cfg.gs.densification_interval = min(cfg.gs.densification_interval, max(a.densify_end // 4, 1))
    if a.max_iterations is not None:
        cfg.gs.max_iterations = a.max_iterations
    if a.interval is not None:
        cfg.admm.consensus_interval = a.interval
    with tempfile.TemporaryDirectory() as tmp:
        views = aerial_views(a.points, 2 * a.mx, 2 * a.my, a.width, a.height)
        scenes = split_scene(views, a.mx, a.my, tmp, dev)
    r = run(cfg, scenes[rank], device=dev)
    if rank == 0:
        print(json.dumps({"blocks": world, "num_global": r.entry.num_global, "shared": r.consensus.num_shared,
                          "rounds": len(r.runner.logs), "seconds": r.seconds,
                          "primal": [sum(lg.primal.values()) for lg in r.runner.logs]}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
