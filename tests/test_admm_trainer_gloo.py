"""The ADMM block-trainer loop (dogs_amd.admm_trainer) over torch.distributed (gloo, world size 2, 4 and 8, CPU) against the
single-process sequential restatement of the same split (SequentialADMM: both blocks in one process, consensus by an
in-process sum) -- 3 rounds of local iterations, consensus, dual update, residuals and penalty adaptation gated by
stop_adapt_iter (master_gaussian_trainer.py:665-728, slave_gaussian_trainer.py:100-207).

The local iteration is a torch-only stand-in (a quadratic data term per block, plain gradient steps) carrying the
trainer's ADMM pieces unchanged: the penalty enters as the proximal gradient coef ((x + u) - z) of ADMMBlockState.prox,
exactly as the GPU trainer folds it into SparseGaussianAdam."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WIDTHS = (3, 3, 45, 3, 4, 1)
N_BLOCK, SHARED = 40, 0.25
ROUNDS, INTERVAL = 3, 5


def _cfg():
    from dogs_amd.admm import ADMMConfig
    # adapt in rounds 1-2 (iterations start+5, start+10 <= stop_adapt_iter), not in round 3
    return ADMMConfig(consensus_interval=INTERVAL, stop_adapt_iter=1000 + 2 * INTERVAL,
                      alpha_xyz=3e3, alpha_fdc=3e3, alpha_fr=3e3, alpha_s=3e3, alpha_q=3e3, alpha_o=3e3)


def _block(k, world=2):
    """World 2: block k of a 2-block chain (rows shared with block k-1 start equal to its values).  World 4 / 8: a grid-like
    cover -- 30 rows of its own, 5 shared with the next block (count 2), 10 central rows shared by all (count = world),
    and 4 rows shared by blocks 0-2 (count 3).  Per-block data targets."""
    from dogs_amd.admm_trainer import chain_block_indices
    if world == 2:
        gidx, stride, _ = chain_block_indices(k, N_BLOCK, SHARED)
        ng = stride + N_BLOCK
    else:
        ng = 30 * world + 14
        parts = [torch.arange(30 * k, 30 * k + 30), torch.arange(30 * ((k + 1) % world), 30 * ((k + 1) % world) + 5),
                 torch.arange(30 * world, 30 * world + 10)]
        if k < 3:
            parts.append(torch.arange(30 * world + 10, 30 * world + 14))
        gidx = torch.unique(torch.cat(parts))
    g = torch.Generator().manual_seed(7)
    glob = [torch.randn((ng, w), generator=g) for w in WIDTHS]    # the global scene of all blocks
    params = tuple(t[gidx].clone() for t in glob)
    gt = torch.Generator().manual_seed(50 + k)
    targets = tuple(torch.randn(p.shape, generator=gt) for p in params)
    return gidx, params, targets, ng


def _toy_step(params, state, targets, lr=0.5):
    """One local iteration: grad of 0.5 sum_p mean((x - t)^2) plus the ADMM proximal gradient, gradient step."""
    def step():
        prox = state.prox(params)
        from dogs_amd.admm_trainer import GROUP_OF
        from dogs_amd.admm import PARAM_NAMES
        with torch.no_grad():
            for n, x, t in zip(PARAM_NAMES, params, targets):
                u, z, coef = prox[GROUP_OF[n]]
                g = (x - t) / x.numel() + coef * ((x + u) - z)
                x.sub_(lr * x.numel() ** 0.5 * g)
    return step


def _sequential(world=2):
    from dogs_amd.admm_trainer import ADMMBlockState, SequentialADMM
    cfg = _cfg()
    blocks = [_block(k, world) for k in range(world)]
    states, steps, fns = [], [], []
    for gidx, params, targets, ng in blocks:
        st = ADMMBlockState(params, ng, cfg)
        states.append(st)
        steps.append(_toy_step(params, st, targets))
        fns.append(lambda p=params: p)
    seq = SequentialADMM(steps, states, fns, [b[0] for b in blocks], blocks[0][3], cfg, 1000, torch.device("cpu"))
    for _ in range(ROUNDS):
        seq.round()
    return blocks, states, seq


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dogs_amd.admm import BlockConsensus
        from dogs_amd.admm_trainer import ADMMBlockState, ADMMRunner
        cfg = _cfg()
        gidx, params, targets, ng = _block(rank, world)
        st = ADMMBlockState(params, ng, cfg)
        cons = BlockConsensus(gidx, ng, device=torch.device("cpu"))
        if world >= 4:
            vc = cons.visibility_count
            assert int((vc == 2).sum()) > 0 and int((vc == 3).sum()) > 0 and int((vc == world).sum()) > 0
        run = ADMMRunner(lambda: params, st, cons, _toy_step(params, st, targets), cfg, 1000)
        for _ in range(ROUNDS):
            run.round()
        ref_blocks, ref_states, seq = _sequential(world)
        assert [lg.adapted for lg in run.logs] == [True, True, False]
        assert [lg.adapted for lg in seq.logs] == [True, True, False]
        for lg, lr_ in zip(run.logs, seq.logs):
            assert lg.iteration == lr_.iteration
            assert lg.primal == lr_.primal and lg.dual == lr_.dual and lg.rho == lr_.rho
        assert any(lg.primal["xyz"] > 0 for lg in run.logs)
        # the penalty parameters moved while adaptation was on, and froze after stop_adapt_iter
        from dogs_amd.admm import initial_rho
        assert run.logs[1].rho != initial_rho(cfg, ng)
        assert run.logs[2].rho == run.logs[1].rho
        # the consensus adds a shared row's copies in block order on every rank, as the sequential restatement does:
        # three rounds of steps stay bit-identical, whatever the count
        for x, y in zip(params, ref_blocks[rank][1]):
            assert torch.equal(x, y)
        for a, b in zip(st.u + st.z, ref_states[rank].u + ref_states[rank].z):
            assert torch.equal(a, b)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_admm_trainer_loop_gloo_matches_sequential(world):
    mp.spawn(_worker, args=(world, _free_port()), nprocs=world, join=True)


def test_sequential_split_consensus_matches_master_average():
    """InProcessConsensus = the master's gaussian_splat_consensus (global zeros, plus_gaussians at each block's
    indices, average by visibility_count; gaussian_splat_model.py:316-340) read back at each block's indices."""
    from dogs_amd.admm_trainer import InProcessConsensus
    blocks = [_block(k) for k in range(2)]
    ng = blocks[0][3]
    cons = InProcessConsensus([b[0] for b in blocks], ng, torch.device("cpu"))
    zs = cons.consensus([b[1] for b in blocks])
    cnt = torch.zeros(ng)
    sums = [torch.zeros(ng, w) for w in WIDTHS]
    for gidx, ps, _, _ in blocks:
        cnt.index_add_(0, gidx, torch.ones(gidx.numel()))
        for s, p in zip(sums, ps):
            s.index_add_(0, gidx, p)
    for (gidx, ps, _, _), z in zip(blocks, zs):
        for k, zz in enumerate(z):
            assert torch.equal(zz, (sums[k] / cnt[:, None])[gidx])
