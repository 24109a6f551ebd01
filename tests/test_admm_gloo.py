"""ADMM block consensus over torch.distributed (gloo, world_size 2, 4 and 8, CPU; at 4 and 8 some Gaussians sit in 3 or
more blocks) vs a single-process restatement of the
reference master's gather/average/scatter (master_gaussian_trainer.py:459-555, gaussian_splat_model.py:316-340),
dual update (slave_gaussian_trainer.py:100-121), residuals (master :396-456) and penalty adaptation (:337-377)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WIDTHS = (3, 3, 45, 3, 4, 1)
N_GLOBAL = 97


def _block(rank, world):
    """Deterministic block data: overlapping global-index sets covering every Gaussian."""
    g = torch.Generator().manual_seed(100 + rank)
    base = torch.arange(rank, N_GLOBAL, world)                       # disjoint cover
    extra = torch.randperm(N_GLOBAL, generator=g)[:30]                # shared Gaussians
    idx = torch.unique(torch.cat([base, extra]))
    params = tuple(torch.randn((idx.numel(), w), generator=g) for w in WIDTHS)
    return idx, params


def _reference(world):
    blocks = [_block(k, world) for k in range(world)]
    cnt = torch.zeros(N_GLOBAL)
    sums = [torch.zeros(N_GLOBAL, w) for w in WIDTHS]
    for idx, ps in blocks:
        cnt.index_add_(0, idx, torch.ones(idx.numel()))
        for s, p in zip(sums, ps):
            s.index_add_(0, idx, p)
    z = [s / cnt[:, None] for s in sums]
    return blocks, cnt, z


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dogs_amd.admm import ADMMConfig, BlockConsensus, adapt_rho, admm_penalty, initial_rho
        blocks, cnt, zref = _reference(world)
        idx, params = blocks[rank]
        bc = BlockConsensus(idx, N_GLOBAL, device=torch.device("cpu"))
        assert torch.equal(bc.visibility_count.float(), cnt)
        if world >= 4:
            assert int((cnt >= 3).sum()) > 0 and int((cnt == 4).sum()) > 0
        # owner = the lowest rank holding the Gaussian: every global row is owned exactly once over the ranks
        owned = torch.zeros(N_GLOBAL, dtype=torch.int64)
        owned[idx[bc.owned]] = 1
        dist.all_reduce(owned)
        assert bool((owned == 1).all())
        lowest = torch.full((N_GLOBAL,), world, dtype=torch.int64)
        for k in range(world):
            i, _ = _block(k, world)
            lowest[i] = torch.minimum(lowest[i], torch.full_like(i, k))
        assert torch.equal(bc.owned, lowest[idx] == rank)
        z = bc.consensus(params)
        # bit-identical for every count: the ranks' copies are added in block order onto zeros and divided by the
        # count, the master's reinitialize / plus_gaussians / average_gaussians arithmetic
        for zi, zr in zip(z, zref):
            assert torch.equal(zi, zr[idx])
        # Gaussians held by one block: z == x exactly, so their dual never moves
        solo = cnt[idx] == 1
        for zi, p in zip(z, params):
            assert torch.equal(zi[solo], p[solo])
        cfg = ADMMConfig()
        rho = initial_rho(cfg, N_GLOBAL)
        duals = [torch.zeros_like(p) for p in params]
        bc.update_duals(duals, params, z, cfg.over_relaxation_coeff)
        for u, p, zi in zip(duals, params, z):
            torch.testing.assert_close(u, 1.5 * (p - zi))
        # a second round with moved parameters -> residuals against the single-process restatement
        params2 = tuple(p + 0.01 * (k + 1) for k, p in enumerate(params))
        z2 = bc.consensus(params2)
        primal, dual = bc.residuals(params2, z2, z, rho)
        blocks2 = [(i, tuple(p + 0.01 * (k + 1) for k, p in enumerate(ps))) for i, ps in blocks]
        z2ref = [zr + 0.01 * (k + 1) for k, zr in enumerate(zref)]
        for k, name in enumerate(("xyz", "fdc", "fr", "s", "q", "o")):
            pr = sum(torch.nn.functional.mse_loss(z2ref[k][i], ps[k]).item() for i, ps in blocks2)
            du = rho[name] * torch.nn.functional.mse_loss(zref[k], z2ref[k]).item()
            assert abs(primal[name] - pr) <= 1e-6 * max(1.0, abs(pr))
            assert abs(dual[name] - du) <= 1e-6 * max(1e-12, abs(du)) + 1e-12
        rho2 = adapt_rho(rho, primal, dual, cfg)
        for name in rho:
            assert rho2[name] in (rho[name], rho[name] * cfg.tau_inc, rho[name] / cfg.tau_dec)
        pen = admm_penalty(params2, duals, z2, rho)
        assert torch.isfinite(pen)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_consensus_gloo_matches_single_process(world):
    mp.spawn(_worker, args=(world, _free_port()), nprocs=world, join=True)


def test_consensus_single_rank_is_identity():
    from dogs_amd.admm import BlockConsensus
    idx, params = _block(0, 1)
    bc = BlockConsensus(idx, N_GLOBAL, device=torch.device("cpu"))
    z = bc.consensus(params)
    for zi, p in zip(z, params):
        assert torch.equal(zi, p)


def test_ordered_sum_is_block_order_sum_divided_by_count():
    """count-2 rows of a two-term sum, count-3 rows whose float association matters: both equal the block-order sum /
    count exactly, and differ from the reversed order / the reciprocal product somewhere (so the check has teeth)."""
    mp.spawn(_ordered_worker, args=(3, _free_port()), nprocs=3, join=True)


def _ordered_worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dogs_amd.admm import ordered_sum_average
        S, D = 1001, 7
        g = torch.Generator().manual_seed(3)
        xs = [torch.randn((S, D), generator=g) * (10.0 ** torch.randint(-3, 4, (S, 1), generator=g)) for _ in range(3)]
        count = torch.full((S, 1), 3.0)
        count[::2] = 2.0
        xs[2][::2] = 0.0                                   # even rows: held by ranks 0 and 1 only
        got = ordered_sum_average(xs[rank].clone(), count, world, rank)
        ref = ((torch.zeros(S, D) + xs[0]) + xs[1]) + xs[2]
        assert torch.equal(got, ref / count)
        assert not torch.equal(got[1::2], (((xs[2] + xs[1]) + xs[0]) / count)[1::2])
        assert not torch.equal(got, ref * (1.0 / count))
    finally:
        dist.destroy_process_group()
