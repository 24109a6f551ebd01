"""Multi-rank ADMM on device tensors, rehearsed with two gloo ranks sharing the one GPU of the test box (RCCL needs
one GPU per rank; the driver's 8-GPU run uses it), plus the ADMM phase entry from a real block split.

* Two ranks run ADMMRunner over real BlockTrainers (native dg_train_step local iterations, 20% of the Gaussians
  shared between the blocks) for two consensus rounds; each rank's parameters, duals and residual logs equal the
  single-process SequentialADMM of the same split (the north star's single-GPU baseline).
* The phase entry from the COLMAP fixture: views -> Grid2D split of the cameras and of the points (bounding boxes,
  world-to-OBB transform) -> block folders (export_blocks) -> per-block models from the block points
  (init_from_colmap_pcd) -> enter_admm_phase_sequential with the HIP kernels (count renders over every block's
  cameras, box membership, prune compaction) equals the same entry with the box tests and compaction restated on the
  CPU, bit for bit; then block trainers from the entries run one consensus round; and two gloo ranks sharing the GPU
  (enter_admm_phase, one block each) reach exactly the single-process entries.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden", "colmap")
N, W, H, VIEWS, SHARED = 20_000, 400, 304, 4, 0.2


def _cfg():
    from dogs_amd.admm import ADMMConfig
    return ADMMConfig(consensus_interval=20, stop_adapt_iter=10 ** 9)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dogs_amd.admm_trainer import distributed_trainer
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        tr, cons, run = distributed_trainer(rank, world, N, W, H, VIEWS, SHARED, dev, admm=_cfg())
        logs = [run.round() for _ in range(2)]
        torch.save({"params": [p.detach().cpu() for p in tr.param_tuple()], "u": [u.cpu() for u in tr.admm.u],
                    "primal": [lg.primal for lg in logs], "dual": [lg.dual for lg in logs],
                    "rho": [lg.rho for lg in logs], "shared": cons.num_shared},
                   os.path.join(out_dir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_two_ranks_match_sequential(hip_device):
    from dogs_amd.admm_trainer import sequential_trainer
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rank_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        got = [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(2)]
    blocks, seq = sequential_trainer(2, N, W, H, VIEWS, SHARED, hip_device, admm=_cfg())
    logs = [seq.round() for _ in range(2)]
    assert got[0]["shared"] == got[1]["shared"] == seq.cons.num_shared > 0
    for r in range(2):
        for a, b in zip(got[r]["params"], blocks[r].param_tuple()):
            torch.testing.assert_close(a, b.detach().cpu(), rtol=1e-6, atol=1e-7)
        for a, b in zip(got[r]["u"], blocks[r].admm.u):
            torch.testing.assert_close(a, b.cpu(), rtol=1e-6, atol=1e-9)
        for k, lg in enumerate(logs):
            for n in lg.primal:
                assert got[r]["primal"][k][n] == pytest.approx(lg.primal[n], rel=1e-6, abs=1e-15)
                assert got[r]["dual"][k][n] == pytest.approx(lg.dual[n], rel=1e-6, abs=1e-15)
            assert got[r]["rho"][k] == lg.rho
    assert sum(logs[-1].primal.values()) > 0


# ---- the phase entry from the COLMAP fixture

def _split(tmp):
    """COLMAP fixture -> (views, camera blocks (RasterCameras), point boxes, expanded point boxes, transform,
    block point sets)."""
    from dogs_amd.blockio import colmap_views, export_blocks
    from dogs_amd.blocksplit import cluster_image_in_grid, cluster_points_in_grid
    v = colmap_views(GOLD, factor=8, scale=False)
    n_img = len(v["image_names"])
    ids, _, _, _ = cluster_image_in_grid(v["camtoworlds"], tmp, list(range(n_img)), [1.4, 1.4, 1.4],
                                         v["image_index_to_image_id"], num_blocks=2, mx=2, my=1)
    bb, ebb, T = cluster_points_in_grid(v["points3d"], v["colors"], tmp, [1.4, 1.4, 1.4], num_blocks=2, mx=2, my=1)
    ds = export_blocks(tmp, v, ids)
    return v, ds, [b.reshape(-1) for b in bb], [b.reshape(-1) for b in ebb], T


def _block_models(v, ebb, T, dev):
    from dogs_amd.blocksplit import points_in_bbox2D
    from dogs_amd.gaussian_model import GaussianSplatModel
    models = []
    for b in ebb:
        sel = points_in_bbox2D(v["points3d"][:, :2], b.reshape(2, 3), T)
        m = GaussianSplatModel(3, 0.01, dev)
        m.init_from_colmap_pcd(v["points3d"][sel], v["colors"][sel] / 255.0)
        m.active_sh_degree = 3
        models.append(m)
    return models


def _cpu_box_kernels():
    from dogs_amd.admm_phase import PhaseKernels
    from oracle.blocksplit_oracle import points_in_bbox2D

    class Mixed(PhaseKernels):   # HIP count renders; box tests and compaction restated on the CPU
        def members(self, xy, boxes, transform):
            return [torch.from_numpy(points_in_bbox2D(xy.cpu().numpy(), np.asarray(b).reshape(2, 3), transform))
                    .to(xy.device) for b in boxes]

        def prune(self, model, mask):
            model.extract_sub_gaussians(torch.nonzero(~mask).squeeze(-1))
    return Mixed()


def _entry_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dogs_amd.admm_phase import PhaseConfig, enter_admm_phase
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        with tempfile.TemporaryDirectory() as tmp:
            v, ds, bb, ebb, T = _split(tmp)
        models = _block_models(v, ebb, T, dev)
        cams = [[c.raster_camera(dev) for c in d.cameras] for d in ds]
        e = enter_admm_phase(models[rank], cams, bb, ebb, T, PhaseConfig())
        torch.save({"gidx": e.global_indices.cpu(), "vis": e.visibility_count.cpu(), "rho": e.rho_gaussians,
                    "params": [t.detach().cpu() for t in e.model.get_all_properties()]},
                   os.path.join(out_dir, f"entry{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_phase_entry_from_colmap_split(hip_device, tmp_path):
    from dogs_amd.admm import ADMMConfig
    from dogs_amd.admm_phase import PhaseConfig, PhaseKernels, enter_admm_phase_sequential
    from dogs_amd.admm_trainer import BlockTrainer, SequentialADMM
    dev = hip_device
    v, ds, bb, ebb, T = _split(str(tmp_path))
    assert len(ds) == 2 and all(len(d) > 0 for d in ds)
    cams = [[c.raster_camera(dev) for c in d.cameras] for d in ds]
    entries = enter_admm_phase_sequential(_block_models(v, ebb, T, dev), cams, bb, ebb, T, PhaseConfig(),
                                          PhaseKernels())
    ref = enter_admm_phase_sequential(_block_models(v, ebb, T, dev), cams, bb, ebb, T, PhaseConfig(),
                                      _cpu_box_kernels())
    for e, r in zip(entries, ref):
        assert torch.equal(e.global_indices.cpu(), r.global_indices.cpu())
        assert torch.equal(e.visibility_count, r.visibility_count)
        assert e.rho_gaussians == r.rho_gaussians
        for a, b in zip(e.model.get_all_properties(), r.model.get_all_properties()):
            assert torch.equal(a.detach(), b.detach())
    assert entries[0].rho_gaussians >= entries[0].num_global > 0   # pruned count, before the expanded-box selection
    vis = entries[0].visibility_count
    assert int((vis >= 2).sum()) > 0, "the expanded boxes should share Gaussians"
    # block trainers from the entries, one consensus round
    cfg = ADMMConfig(consensus_interval=5)
    g = torch.Generator().manual_seed(0)
    trainers = []
    for b, e in enumerate(entries):
        imgs = [torch.rand((3, c.height, c.width), generator=g).to(dev) for c in cams[b]]
        trainers.append(BlockTrainer(e.raw(), cams[b], imgs, e.num_global, cfg, device=dev, seed=b,
                                     rho_gaussians=e.rho_gaussians))
    seq = SequentialADMM([t.local_step for t in trainers], [t.admm for t in trainers],
                         [t.param_tuple for t in trainers], [e.global_indices for e in entries],
                         entries[0].num_global, cfg, trainers[0].iteration, dev)
    lg = seq.round()
    assert seq.cons.num_shared == int((vis >= 2).sum())
    assert torch.equal(seq.cons.visibility_count.to(torch.int64), vis)
    assert all(np.isfinite(x) for x in lg.primal.values()) and sum(lg.primal.values()) > 0
    assert all(bool(torch.isfinite(p).all()) for t in trainers for p in t.param_tuple())
    # the distributed entry (two gloo ranks sharing the GPU) reaches the same entries
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_entry_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        got = [torch.load(os.path.join(d, f"entry{r}.pt"), weights_only=True) for r in range(2)]
    for r, e in enumerate(entries):
        assert torch.equal(got[r]["gidx"], e.global_indices.cpu())
        assert torch.equal(got[r]["vis"], e.visibility_count.cpu())
        assert got[r]["rho"] == e.rho_gaussians
        for a, b in zip(got[r]["params"], e.model.get_all_properties()):
            assert torch.equal(a, b.detach().cpu())
