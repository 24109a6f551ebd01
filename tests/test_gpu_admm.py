"""The ADMM block trainer on the GPU (dogs_amd.admm_trainer):

* the penalty folded into SparseGaussianAdam (dg_adam_update_groups_prox) gives the same Adam moments as the
  reference's route -- 0.5 rho mse(x + u, z) added to the loss (slave_gaussian_trainer.py:161-202), differentiated by
  torch autograd, then the plain sparse Adam step -- within 1e-5 relative (fp32 rounding of the two gradient sums);
* consensus, dual update, residuals and the penalty value on device tensors equal the same code on the host (1e-6);
* a short sequential ADMM run (2 blocks, 2 rounds) on one GPU stays finite and moves the penalty parameters.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _small_block(dev, k=0, blocks=2, n=4000, W=192, H=128, native=False, views=1):
    from dogs_amd.admm import ADMMConfig
    from dogs_amd.admm_trainer import TrainConfig, make_block
    return make_block(k, blocks, n, W, H, views, 0.25, dev, seed=77, admm=ADMMConfig(consensus_interval=3),
                      cfg=TrainConfig(), native=native)


def _perturb_state(tr, seed):
    g = torch.Generator().manual_seed(seed)
    st = tr.admm
    st.u = tuple((0.01 * torch.randn(p.shape, generator=g)).to(p.device) for p in tr.param_tuple())
    st.z = tuple((p.detach().cpu() + 0.02 * torch.randn(p.shape, generator=g)).to(p.device)
                 for p in tr.param_tuple())
    st.rho = {k: v * 1e3 for k, v in st.rho.items()}   # make the penalty matter against the image terms


def test_prox_adam_matches_autograd_penalty(hip_device):
    from dogs_amd.admm import PARAM_NAMES, admm_penalty
    a, _, _ = _small_block(hip_device)
    b, _, _ = _small_block(hip_device)
    _perturb_state(a, 3)
    _perturb_state(b, 3)
    a.local_step()                      # penalty as the proximal gradient inside the Adam launch
    # reference route on b: the same iteration with the penalty in the loss, then the plain sparse Adam step
    b.iteration += 1
    for g in b.opt.param_groups:
        if g["name"] == "xyz":
            g["lr"] = b.xyz_lr(b.iteration)
    p = b.params
    k = b._next_view()
    gt = b.images[k]
    m2d = torch.zeros_like(p["xyz"], requires_grad=True)
    opac, scales, rots = b.activate(p["opacity"], p["scaling"], p["quaternion"])
    img, radii, _ = b.rasts[k](means3D=p["xyz"], means2D=m2d, opacities=opac, dc=p["features_dc"],
                               shs=p["features_rest"], scales=scales, rotations=rots)
    img, l1 = b.clamp_l1(img, gt)
    ssim = b.fused_ssim(img.unsqueeze(0), gt.unsqueeze(0))
    c = b.cfg
    loss = (1.0 - c.lambda_dssim) * l1 + c.lambda_dssim * (1.0 - ssim) + c.lambda_scale * scales.prod(dim=1).mean()
    loss = loss + admm_penalty(b.param_tuple(), list(b.admm.u), b.admm.z, b.admm.rho)
    loss.backward()
    vis = radii > 0
    b.opt.step(vis, radii.shape[0])
    assert int(vis.sum()) > 100
    for n in PARAM_NAMES:
        ma = a.opt.state[a.params[n]]["exp_avg"]
        mb = b.opt.state[b.params[n]]["exp_avg"]
        err = float((ma - mb).norm() / mb.norm())
        assert err < 1e-5, (n, err)
        # rows outside the view: untouched by either route (SparseGaussianAdam ignores their gradient)
        assert float(ma[~vis].abs().max()) == 0.0
        torch.testing.assert_close(a.params[n].detach(), b.params[n].detach(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("n,W,H", [(4000, 192, 128), (20000, 400, 304)])
def test_native_step_matches_autograd(hip_device, n, W, H):
    """dg_train_step (one C call: activations, rasterizer, clamp/L1, SSIM, loss gradient, backward, scale regulariser,
    Adam with the ADMM proximal gradient) against the autograd route of the same iteration, three iterations with a
    perturbed ADMM state: radii equal, Adam moments within 1e-5 relative, parameters within 1e-5, loss within 1e-5
    (fp32 summation orders differ: the loss partial sums, the regulariser's product gradient)."""
    from dogs_amd.admm import PARAM_NAMES
    a, _, _ = _small_block(hip_device, n=n, W=W, H=H, native=True)
    b, _, _ = _small_block(hip_device, n=n, W=W, H=H, native=False)
    _perturb_state(a, 9)
    _perturb_state(b, 9)
    for _ in range(3):
        a.local_step()
        b.local_step()
        assert torch.equal(a.last_radii, b.last_radii)
        torch.testing.assert_close(a.last_loss, b.last_loss, rtol=1e-5, atol=1e-7)
    assert int((a.last_radii > 0).sum()) > 100
    for nm in PARAM_NAMES:
        for key in ("exp_avg", "exp_avg_sq"):
            ma = a.opt.state[a.params[nm]][key]
            mb = b.opt.state[b.params[nm]][key]
            err = float((ma - mb).norm() / mb.norm())
            assert err < 1e-5, (nm, key, err)
        torch.testing.assert_close(a.params[nm].detach(), b.params[nm].detach(), rtol=1e-5, atol=1e-6)


def test_device_consensus_residuals_penalty_match_host(hip_device):
    from dogs_amd.admm import RHO_NAMES, ADMMConfig, initial_rho
    from dogs_amd.admm_trainer import ADMMBlockState, InProcessConsensus, chain_block_indices
    cfg = ADMMConfig()
    g = torch.Generator().manual_seed(11)
    n, f = 500, 0.3
    idx = [chain_block_indices(k, n, f)[0] for k in range(3)]
    ng = int(idx[-1][-1]) + 1
    widths = (3, 3, 45, 3, 4, 1)
    host = [tuple(torch.randn((n, w), generator=g) for w in widths) for _ in range(3)]
    out = {}
    for dev in (torch.device("cpu"), hip_device):
        ps = [tuple(t.to(dev) for t in b) for b in host]
        cons = InProcessConsensus([i.to(dev) for i in idx], ng, dev)
        sts = [ADMMBlockState(p, ng, cfg) for p in ps]
        moved = [tuple(t + 0.05 * (j + 1) for j, t in enumerate(p)) for p in ps]
        zs = cons.consensus(moved)
        for st, p, z in zip(sts, moved, zs):
            st.update_duals(p, z)
        rho = initial_rho(cfg, ng)
        primal, dual = cons.residuals(moved, [s.z for s in sts], [s.z_prev for s in sts], rho)
        pen = [float(s.penalty(p)) for s, p in zip(sts, moved)]
        out[dev.type] = (zs, [s.u for s in sts], primal, dual, pen)
    zc, uc, pc, dc, penc = out["cpu"]
    zg, ug, pg, dg, peng = out["cuda"]
    for a, b in zip(zc + uc, zg + ug):
        for x, y in zip(a, b):
            torch.testing.assert_close(x, y.cpu(), rtol=1e-6, atol=1e-6)
    for k in RHO_NAMES:
        assert abs(pc[k] - pg[k]) <= 1e-6 * max(abs(pc[k]), 1e-12)
        assert abs(dc[k] - dg[k]) <= 1e-6 * max(abs(dc[k]), 1e-12)
        assert pc[k] > 0.0 and dc[k] > 0.0
    np.testing.assert_allclose(penc, peng, rtol=1e-5)


def test_sequential_admm_two_blocks_gpu(hip_device):
    from dogs_amd.admm import ADMMConfig
    from dogs_amd.admm_trainer import sequential_trainer
    cfg = ADMMConfig(consensus_interval=3, stop_adapt_iter=30003)
    blocks, seq = sequential_trainer(2, 3000, 128, 96, 1, 0.25, hip_device, admm=cfg, seed=5)
    logs = [seq.round() for _ in range(2)]
    assert [lg.adapted for lg in logs] == [True, False]
    for b in blocks:
        assert torch.isfinite(b.last_loss)
        assert all(torch.isfinite(p).all() for p in b.param_tuple())
        assert torch.isfinite(b.penalty())
    assert logs[0].primal["xyz"] > 0.0


@pytest.mark.parametrize("n,W,H", [(4000, 192, 128), (20000, 400, 304)])
def test_native_step_folded_update_bitwise(hip_device, monkeypatch, n, W, H):
    """dg_train_step's default route -- the activations' backward folded into the update, and the chunks touching no
    binned row skipping the (zero) gradient reads -- gives bit-identical parameters, moments and densification
    statistics to the unfused route (k_activate_bwd, then the plain update: DG_TRAIN_UNFUSED=1), three iterations with
    a perturbed ADMM state (proximal gradient on).  So does the overlapped route (NativeTrainStep(overlap=True): the
    f_dc / f_rest update of each step on a side stream, beside the next step's forward until its emission)."""
    from dogs_amd.admm import PARAM_NAMES
    from dogs_amd.train_step import NativeTrainStep
    routes = {"folded": None, "unfused": "DG_TRAIN_UNFUSED", "overlap": None}
    tr, stats = {}, {}
    for name in routes:
        t, _, _ = _small_block(hip_device, n=n, W=W, H=H, native=True)
        _perturb_state(t, 9)
        rows = int(t.params["xyz"].shape[0])
        stats[name] = {k: torch.zeros(rows, dtype=torch.float32, device=hip_device)
                       for k in ("max_radii2D", "grad_accum", "denom")}
        c = t.cfg
        t._nts = NativeTrainStep({nm: t.params[nm] for nm in PARAM_NAMES}, t.opt, t.cameras, t.images, c.sh_degree,
                                 c.lambda_dssim, c.lambda_scale, torch.tensor(c.background, dtype=torch.float32),
                                 hip_device, stats=stats[name], overlap=name == "overlap")
        tr[name] = t
    assert tr["overlap"]._nts.overlap
    for it in range(4):
        for name, env in routes.items():
            monkeypatch.delenv("DG_TRAIN_UNFUSED", raising=False)
            if env:
                monkeypatch.setenv(env, "1")
            tr[name].local_step()
        if it != 1:  # one round left pending across the next step's forward without a device sync in between
            torch.cuda.synchronize()
    tr["overlap"]._nts.sync()
    torch.cuda.synchronize()
    monkeypatch.delenv("DG_TRAIN_UNFUSED", raising=False)
    ref = tr["unfused"]
    vis = ref.last_radii > 0
    assert int(vis.sum()) > 100 and int((~vis).sum()) > 0
    for name in ("folded", "overlap"):
        t = tr[name]
        assert torch.equal(t.last_radii, ref.last_radii)
        for nm in PARAM_NAMES:
            assert torch.equal(t.params[nm].detach(), ref.params[nm].detach()), (name, nm)
            for key in ("exp_avg", "exp_avg_sq"):
                assert torch.equal(t.opt.state[t.params[nm]][key], ref.opt.state[ref.params[nm]][key]), (name, nm, key)
        for key, v in stats["unfused"].items():
            assert torch.equal(stats[name][key], v), (name, key)
        assert float(stats[name]["denom"].max()) >= 1.0 and float(stats[name]["grad_accum"].max()) > 0.0
