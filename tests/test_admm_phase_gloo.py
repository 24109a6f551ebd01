"""The ADMM phase entry (dogs_amd.admm_phase: fuse_local_gaussians without the RPC master,
master_gaussian_trainer.py:37-172, 557-618) over torch.distributed (gloo, world size 2, 3, 4 and 8, CPU; at world 3
the middle block has no cameras, world 8 is a 2 x 4 grid).

The device operations (count renders, box membership, prune compaction) are replaced by CPU restatements
(`CPUKernels`), so this checks the distributed plumbing and the lifecycle order:
  * every rank's entry equals the single-process entry (enter_admm_phase_sequential) bit for bit -- the gathered and
    fused model, the importance (folded down the rank chain in the reference's camera order), the pruned set, the
    expanded-box split, visibility_count and the penalty denominator;
  * the single-process entry equals a plain restatement of the reference's own steps written here from its source
    (clip to the original boxes, concatenate, prune_list over the concatenated camera list popped from the end,
    calculate_v_imp_score, prune_gaussians(0.4 p), select_gaussians_in_each_block).
World 4 is a 2 x 2 grid whose expanded boxes overlap at the centre, so Gaussians there sit in 3 or 4 blocks (count
3-4, owner = the lowest of up to four ranks).
The HIP versions of the three operations are checked on the GPU (tests/test_gpu_admm_dist.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
T = np.array([[0.8, -0.6, 0.3], [0.6, 0.8, -0.2], [0.0, 0.0, 1.0]])   # world -> OBB (a rotation + shift)
# world 2: two halves; world 4: a 2 x 2 grid (boxes in the OBB frame [x0, y0, z0, x1, y1, z1], expanded by 1)
GRIDS = {
    2: [(-5.0, -5.0, 0.0, 5.0), (0.0, -5.0, 5.0, 5.0)],
    4: [(-5.0, -5.0, 0.0, 0.0), (0.0, -5.0, 5.0, 0.0), (-5.0, 0.0, 0.0, 5.0), (0.0, 0.0, 5.0, 5.0)],
    3: [(-6.0, -5.0, -2.0, 5.0), (-2.0, -5.0, 2.0, 5.0), (2.0, -5.0, 6.0, 5.0)],   # block 1 has no cameras
    # world 8: a 2 x 4 grid (the sci-art / MatrixCity block count); cells 2.5 tall, so an expanded box reaches two
    # rows away and a Gaussian near a column border sits in up to six blocks
    8: [(-5.0 + 5.0 * i, -5.0 + 2.5 * j, 5.0 * i, -2.5 + 2.5 * j) for j in range(4) for i in range(2)],
}


def _boxes(world):
    ori = [np.array([x0, y0, -1.0, x1, y1, 1.0]) for x0, y0, x1, y1 in GRIDS[world]]
    exp = [np.array([x0 - 1.0, y0 - 1.0, -1.0, x1 + 1.0, y1 + 1.0, 1.0]) for x0, y0, x1, y1 in GRIDS[world]]
    return ori, exp


def _cameras(world):
    g = torch.Generator().manual_seed(3)
    # world 3: the middle block has no cameras (its rank folds nothing onto the importance chain and passes it on)
    return [[torch.randn(3, generator=g) * 3.0 for _ in range(0 if (world == 3 and b == 1) else 3 + (b % 2))]
            for b in range(world)]


def _block_model(b, world):
    """Block b's model: points around its grid cell (in the OBB frame), so blocks overlap near the cell borders."""
    from dogs_amd.gaussian_model import GaussianSplatModel
    g = torch.Generator().manual_seed(11 + b)
    n = 300 - 20 * b
    m = GaussianSplatModel(3, 0.01, "cpu")
    x0, y0, x1, y1 = GRIDS[world][b]
    obb = torch.stack([x0 + (x1 - x0) * (torch.rand(n, generator=g) * 1.4 - 0.2),
                       y0 + (y1 - y0) * (torch.rand(n, generator=g) * 1.4 - 0.2)], 1).double()
    Ti = torch.from_numpy(np.linalg.inv(T))
    xy = (obb @ Ti[:2, :2].T + Ti[:2, 2]).float()
    xyz = torch.cat([xy, torch.randn(n, 1, generator=g) * 0.3], 1)
    m.init_from_external_properties(xyz, torch.randn(n, 1, 3, generator=g), torch.randn(n, 15, 3, generator=g) * 0.1,
                                    torch.randn(n, 3, generator=g) - 3.0, torch.randn(n, 4, generator=g),
                                    torch.randn(n, 1, generator=g), optimizable=True)
    m.active_sh_degree = 2
    return m


def _cpu_kernels():
    from dogs_amd.admm_phase import PhaseKernels
    from oracle.blocksplit_oracle import points_in_bbox2D

    class CPUKernels(PhaseKernels):
        def camera_importance(self, model, camera, bg):
            xyz = model.get_xyz.detach()
            op = torch.sigmoid(model.get_raw_opacity.detach()).reshape(-1)
            d = ((xyz - camera) ** 2).sum(1)
            cnt = (d < 40.0).to(torch.int32) * (1 + (d.to(torch.int32) % 7))   # integer pixel counts
            return cnt.float() * op

        def members(self, xy, boxes, transform):
            return [torch.from_numpy(points_in_bbox2D(xy.numpy(), np.asarray(b).reshape(2, 3), transform))
                    for b in boxes]

        def prune(self, model, mask):
            model.extract_sub_gaussians(torch.nonzero(~mask).squeeze(-1))
    return CPUKernels()


def _restated(cfg, world):
    """The reference's steps, from its source text, on the same blocks and kernels."""
    from oracle.blocksplit_oracle import points_in_bbox2D
    K = _cpu_kernels()
    ORI, EXP = _boxes(world)
    models = [_block_model(b, world) for b in range(world)]
    rows = []
    for b, m in enumerate(models):              # fuse_block_gaussians :55-83
        keep = torch.from_numpy(points_in_bbox2D(m.get_xyz.detach().numpy()[:, :2], ORI[b].reshape(2, 3), T))
        rows.append([t.detach()[keep] for t in (m._xyz, m._features_dc, m._features_rest, m._scaling,
                                                m._quaternion, m._opacity)])
    fused = [torch.cat([r[i] for r in rows], 0) for i in range(6)]
    from dogs_amd.gaussian_model import GaussianSplatModel
    F = GaussianSplatModel(3, 0.01, "cpu")
    F.init_from_external_properties(*fused)
    F.active_sh_degree = 3
    cameras = [c for cams in _cameras(world) for c in cams]   # prune_gaussians_after_merge: one list
    imp = K.camera_importance(F, cameras.pop(), None)          # prune_list: pop, then += pop ...
    while cameras:
        imp += K.camera_importance(F, cameras.pop(), None)
    volume = torch.prod(torch.exp(F._scaling), dim=1)                       # calculate_v_imp_score
    sv, _ = torch.sort(volume, descending=True)
    v = torch.pow(volume / sv[int(len(volume) * 0.9)], cfg.v_pow) * imp
    s, _ = torch.sort(v, dim=0)                                             # prune_gaussians
    prune = (v <= s[int(0.4 * cfg.prune_percent * (s.shape[0] - 1))]).squeeze()
    kept = [t[~prune] for t in fused]
    n_rho = kept[0].shape[0]
    gi = [torch.from_numpy(points_in_bbox2D(kept[0].numpy()[:, :2], e.reshape(2, 3), T)) for e in EXP]
    cnt = torch.bincount(torch.cat(gi))                                     # select_gaussians_in_each_block
    valid = torch.argwhere(cnt).squeeze(-1)
    kept = [t[valid] for t in kept]
    gi = [torch.from_numpy(points_in_bbox2D(kept[0].numpy()[:, :2], e.reshape(2, 3), T)) for e in EXP]
    vis = torch.bincount(torch.cat(gi))
    return kept, gi, vis, n_rho


def _sequential(cfg, world):
    from dogs_amd.admm_phase import enter_admm_phase_sequential
    ORI, EXP = _boxes(world)
    return enter_admm_phase_sequential([_block_model(b, world) for b in range(world)], _cameras(world), ORI, EXP, T,
                                       cfg, _cpu_kernels())


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dogs_amd.admm_phase import PhaseConfig, enter_admm_phase
        cfg = PhaseConfig(prune_percent=0.5, v_pow=0.1)
        ORI, EXP = _boxes(world)
        e = enter_admm_phase(_block_model(rank, world), _cameras(world), ORI, EXP, T, cfg, _cpu_kernels())
        ref = _sequential(cfg, world)[rank]
        assert torch.equal(e.global_indices, ref.global_indices)
        assert torch.equal(e.visibility_count, ref.visibility_count)
        assert (e.num_global, e.rho_gaussians) == (ref.num_global, ref.rho_gaussians)
        for a, b in zip(e.model.get_all_properties(), ref.model.get_all_properties()):
            assert torch.equal(a.detach(), b.detach())
        for a, b in zip(e.fused.get_all_properties(), ref.fused.get_all_properties()):
            assert torch.equal(a, b)
        assert e.model.active_sh_degree == 3   # the master's degree (max), not the blocks'
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_phase_entry_gloo_matches_single_process(world):
    mp.spawn(_worker, args=(world, _free_port()), nprocs=world, join=True)


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_single_process_entry_matches_reference_steps(world):
    from dogs_amd.admm_phase import PhaseConfig
    cfg = PhaseConfig(prune_percent=0.5, v_pow=0.1)
    entries = _sequential(cfg, world)
    kept, gi, vis, n_rho = _restated(cfg, world)
    assert entries[0].rho_gaussians == n_rho
    assert torch.equal(entries[0].visibility_count, vis)
    assert 0 < n_rho < sum(300 - 20 * b for b in range(world))
    assert int((vis >= 2).sum()) > 0, "the expanded boxes must overlap"
    if world == 4:
        assert int((vis >= 3).sum()) > 0 and int((vis == 4).sum()) > 0, "the grid centre must be shared by 3-4 blocks"
    if world == 8:
        assert int((vis >= 3).sum()) > 0, "a 4-long axis of 2.5-wide cells expanded by 1: rows in >= 3 blocks"
        sizes = {len(e.global_indices) for e in entries}
        assert len(sizes) > 1, "the entry's padded all_gather must see unequal blocks"
    for b in range(world):
        assert torch.equal(entries[b].global_indices, gi[b])
        for a, k in zip(entries[b].model.get_all_properties(), kept):
            assert torch.equal(a.detach(), k[gi[b]])
        assert isinstance(entries[b].model._xyz, torch.nn.Parameter)
        assert entries[b].model.xyz_gradient_accum.shape == (len(gi[b]), 1)
    # fused model = the clipped blocks, pruned
    assert entries[0].fused.num_gaussians == kept[0].shape[0]


def test_all_gather_rows_variable_sizes():
    mp.spawn(_gather_worker, args=(3, _free_port()), nprocs=3, join=True)


def _gather_worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dogs_amd.admm_phase import all_gather_rows
        rows = torch.arange(rank * 5 * 4, dtype=torch.float32).reshape(rank * 5, 4) + 100 * rank
        got = all_gather_rows(rows)
        want = torch.cat([torch.arange(r * 5 * 4, dtype=torch.float32).reshape(r * 5, 4) + 100 * r
                          for r in range(world)], 0)
        assert got.shape == (15, 4) and torch.equal(got, want)
    finally:
        dist.destroy_process_group()


def test_ordered_importance_bounded_lookahead():
    """ordered_importance with no camera rendered ahead of the chain's partial sum, one, and all of them: the same
    bits as prune_list's pop order over the concatenated camera list."""
    mp.spawn(_importance_worker, args=(3, _free_port()), nprocs=3, join=True)


def _importance_worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dogs_amd.admm_phase import ordered_importance
        K = _cpu_kernels()
        fused = _block_model(0, 4)
        cams = _cameras(4)[:world]
        flat = [c for cs in cams for c in cs]
        want = K.camera_importance(fused, flat.pop(), None)
        while flat:
            want += K.camera_importance(fused, flat.pop(), None)
        n = fused.num_gaussians
        for budget in (0, 4 * n, 1 << 30):
            got = ordered_importance(fused, cams, K, None, score_budget_bytes=budget)
            assert torch.equal(got, want), budget
    finally:
        dist.destroy_process_group()
