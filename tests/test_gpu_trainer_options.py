"""The trainer options the reference configs switch on, on the GPU (gaussian_trainer.py:171-183, 232-257, 309-319,
356-401, 478-484; urban3d_admm.yaml: geometry.mask, loss.lambda_mask 0.5, geometry.depth_threshold 0.23;
mipnerf360.yaml: geometry.mask with lambda_mask 0):

* one native step with the appearance mask: its L1 term of clamp(render) * mask, its mean((mask - 1)^2) and its
  dL/dmask equal torch's autograd of the reference's loss expression on the step's own render;
* 20 iterations with the mask (lambda_mask 0.5) and depth_threshold, densification statistics on: the native route
  (dg_train_step + the embedding's backward in torch) and the autograd route (render(depth_threshold=...) +
  F.l1_loss(colors * mask, pixels) + ... + loss.backward(), the reference's expression) follow the same loss
  trajectory and end with the same Gaussians, Adam moments, statistics and embedding parameters;
* depth_threshold changes the statistics exactly as _RasterizeGaussians.backward's scale_tensor (native = autograd,
  and both differ from the unscaled run);
* the trained exposure (its Adam and ExponentialLR) and coarse-to-fine training resolutions run through the autograd
  route with the schedule of the reference.
"""
import copy
import math

import numpy as np
import pytest
import torch

from test_gpu_trainer import _cfg, _normal, _problem

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def test_masked_native_step_matches_torch_loss(hip_device):
    from dogs_amd.masks import AppearanceEmbedding
    from dogs_amd.trainer import GaussianSplatTrainer
    dev = hip_device
    m, cams, gts = _problem(dev, n_true=20_000, n_init=5_000, W=333, H=250, views=2)
    torch.manual_seed(0)
    net = AppearanceEmbedding(len(cams))
    with torch.no_grad():   # a non-trivial embedding row, so the mask differs per view
        net.appearance_embedding.normal_(0.0, 0.5)
    cfg = _cfg(densify_start_iter=10 ** 6, lambda_mask=0.5, mask=True)
    tr = GaussianSplatTrainer(m, cams, gts, cfg, device=dev, seed=0, native=True, appear_embedding=net)
    nts = tr._native_step()
    mask, dmask = tr._masked.forward(1, gts[1], 1)
    nts.step(1, 1e-4, sh_degree=0, mask=mask, dmask=dmask)
    torch.cuda.synchronize()
    colors = nts.image(1).clone()
    mk = mask.detach().clone().requires_grad_(True)
    ld, lm = cfg.lambda_dssim, cfg.lambda_mask
    l1 = torch.nn.functional.l1_loss(colors * mk, gts[1])
    mreg = torch.mean((mk - 1) ** 2.)
    ((1.0 - ld) * l1 + lm * mreg).backward()
    buf = nts.loss_buf.cpu()
    assert float(buf[0]) == pytest.approx(float(l1), rel=2e-6)
    assert float(buf[3]) == pytest.approx(float(mreg), rel=2e-6)
    assert float(buf[3]) > 0.01
    assert _rel(dmask, mk.grad) < 1e-6
    assert float(nts.loss()) == pytest.approx((1 - ld) * float(buf[0]) + ld * (1 - float(buf[1])) + lm * float(buf[3])
                                              + cfg.lambda_scale * float(buf[2]), rel=1e-6)


def _state(tr):
    m = tr.model
    opt = {g["name"]: tr.optimizer.state[g["params"][0]] for g in tr.optimizer.param_groups}
    return ({k: v.detach().clone() for k, v in m.params().items()},
            {k: (v["exp_avg"].clone(), v["exp_avg_sq"].clone()) for k, v in opt.items()},
            (m.max_radii2D.clone(), m.xyz_gradient_accum.clone(), m.denom.clone()))


def test_masked_training_native_matches_autograd(hip_device):
    """20 iterations, mask (lambda_mask 0.5) + depth_threshold + densification statistics: native = autograd bit for
    bit -- parameters, Adam moments, statistics and the embedding's parameters (the masked L1's dL/dmask and
    dL/dcolour, the mask regulariser's and the depth scaling's arithmetic are torch's on both routes; the embedding's
    kernels are deterministic); the logged losses equal to rounding (summed in different orders)."""
    from dogs_amd.masks import AppearanceEmbedding
    from dogs_amd.trainer import GaussianSplatTrainer
    from test_gpu_trainer import _assert_same_state, _route_state
    dev = hip_device
    torch.manual_seed(1)
    net0 = AppearanceEmbedding(4)
    with torch.no_grad():
        net0.appearance_embedding.normal_(0.0, 0.3)
    cfg = _cfg(densify_start_iter=10 ** 6, opacity_reset_interval=10 ** 6, prune_iterations=(), mask=True,
               lambda_mask=0.5, depth_threshold=6.0, sh_increase_interval=7)
    out = []
    for native in (True, False):
        m, cams, gts = _problem(dev, n_true=30_000, n_init=6_000, W=400, H=300, views=4)
        net = copy.deepcopy(net0)
        tr = GaussianSplatTrainer(m, cams, gts, cfg, device=dev, seed=2, native=native, appear_embedding=net,
                                  normal=_normal(dev, 3))
        losses = []
        for _ in range(20):
            tr.train_iteration()
            losses.append(float(tr.loss()))
        assert {lg.route for lg in tr.logs} == {"native" if native else "autograd"}
        out.append((np.array(losses), _route_state(tr), {k: v.detach().clone() for k, v in net.state_dict().items()}))
    (l0, s0, n0), (l1, s1, n1) = out
    print("max rel loss diff", float(np.max(np.abs(l0 - l1) / l1)))
    np.testing.assert_allclose(l0, l1, rtol=1e-5)
    _assert_same_state(s0, s1)
    _assert_same_state(n0, n1)
    assert _rel(n0["appearance_embedding"], net0.state_dict()["appearance_embedding"].to(dev)) > 1e-4   # it trained


@pytest.mark.parametrize("case", ["plain", "mask-depth", "antialiasing", "zero-scaling"])
def test_first_step_native_equals_autograd(hip_device, case):
    """ONE iteration through each route from the same state, SH degree 3 (so f_rest carries gradient): the first Adam
    moment is 0.1 x the raw-parameter gradient and the second 0.001 x its square, so they compare the two routes'
    gradients directly, f_rest included: bit for bit in every row, in every case (tools/first_step_probe.py).  Cases: plain; the appearance mask + lambda_mask 0.5 + depth_threshold
    (urban3d_admm.yaml); texture.anti_aliasing
    (the native step's antialiasing flag); one Gaussian's scaling underflowed to exactly 0, where torch's prod backward
    switches EVERY row to its zero-safe form (the native step reads the activation pass's zero stamp)."""
    from dogs_amd.masks import AppearanceEmbedding
    from dogs_amd.trainer import GaussianSplatTrainer
    dev = hip_device
    kw = dict(densify_start_iter=10 ** 6, opacity_reset_interval=10 ** 6, prune_iterations=(), lambda_scale=0.05)
    if case == "mask-depth":
        kw.update(mask=True, lambda_mask=0.5, depth_threshold=6.0)
    elif case == "antialiasing":
        kw.update(anti_aliasing=True)
    cfg = _cfg(**kw)
    torch.manual_seed(1)
    net0 = AppearanceEmbedding(2)
    with torch.no_grad():
        net0.appearance_embedding.normal_(0.0, 0.3)
    out = []
    for native in (True, False):
        m, cams, gts = _problem(dev, n_true=30_000, n_init=6_000, W=400, H=300, views=2)
        m.active_sh_degree = 3
        with torch.no_grad():   # SH rest, anisotropic scales and turned rotations: every group carries gradient
            gen = torch.Generator(device=dev).manual_seed(4)
            m._features_rest.normal_(0.0, 0.05, generator=gen)
            m._scaling.add_(torch.randn(m._scaling.shape, generator=gen, device=dev) * 0.3)
            m._quaternion.add_(torch.randn(m._quaternion.shape, generator=gen, device=dev) * 0.3)
            if case == "zero-scaling":
                m._scaling[7, 1] = -200.0          # exp(-200) == 0 in float32
        tr = GaussianSplatTrainer(m, cams, gts, cfg, device=dev, seed=2, native=native, normal=_normal(dev, 3),
                                  appear_embedding=copy.deepcopy(net0) if cfg.mask else None)
        tr.train_iteration()
        tr.sync()
        assert [lg.route for lg in tr.logs] == ["native" if native else "autograd"]
        if case == "zero-scaling":
            assert float(torch.exp(m._scaling.detach()).min()) == 0.0
        out.append(_state(tr))
    s0, s1 = out
    # the same kernels and activations with torch's association on both routes, and the masked L1's
    # dL/dmask and dL/dcolour formed as torch's autograd forms them: every group's two Adam moments and the statistics
    # are bit-identical, every row -- the degenerate Gaussian 7 included
    for k in s0[1]:
        assert float(s1[1][k][0].norm()) > 0, k
        for j in (0, 1):
            d = (s0[1][k][j] - s1[1][k][j]).abs().max()
            assert torch.equal(s0[1][k][j], s1[1][k][j]), (k, j, float(d))
    for a, b in zip(s0[2], s1[2]):
        assert torch.equal(a, b)
    if case == "zero-scaling":   # finite, and the zero axis gets exactly no scaling gradient on either route
        for st in (s0, s1):
            assert all(bool(torch.isfinite(v[0][7]).all()) for v in st[1].values())
            assert float(st[1]["scaling"][0][7, 1]) == 0.0


def test_depth_threshold_scales_statistics(hip_device):
    """grad_accum with depth_threshold = the reference's min(1, (depth / thr)^2) scaling of each visible Gaussian's
    screen-space gradient; denom and max_radii2D unchanged; native = autograd."""
    from dogs_amd.trainer import GaussianSplatTrainer
    dev = hip_device
    res = {}
    for native in (True, False):
        for thr in (0.0, 8.0):
            m, cams, gts = _problem(dev, n_true=20_000, n_init=5_000, W=320, H=240, views=1)
            cfg = _cfg(densify_start_iter=10 ** 6, depth_threshold=thr)
            tr = GaussianSplatTrainer(m, cams, gts, cfg, device=dev, seed=0, native=native)
            # the view depth of the rendered (pre-update) positions
            z = (m.get_xyz.detach() @ cams[0].world_to_camera[:3, :3] + cams[0].world_to_camera[3, :3])[:, 2]
            tr.train_iteration()
            tr.sync()
            res[(native, thr)] = (m.xyz_gradient_accum.clone().reshape(-1), m.denom.clone(), z)
    for native in (True, False):
        g0, d0, z = res[(native, 0.0)]
        g1, d1, _ = res[(native, 8.0)]
        assert torch.equal(d0, d1)
        f = torch.minimum(torch.ones_like(z), (z / 8.0) ** 2)
        vis = d0.reshape(-1) > 0
        assert int(vis.sum()) > 100 and bool((f[vis] < 1).any())
        torch.testing.assert_close(g1[vis], g0[vis] * f[vis], rtol=2e-5, atol=1e-9)
    assert _rel(res[(True, 8.0)][0], res[(False, 8.0)][0]) < 1e-4


def test_trained_exposure_and_coarse_to_fine(hip_device):
    from dogs_amd.admm_trainer import ExponentialLR
    from dogs_amd.trainer import GaussianSplatTrainer
    dev = hip_device
    m, cams, gts = _problem(dev, n_true=20_000, n_init=4_000, W=320, H=240, views=3)
    for k, c in enumerate(cams):
        c.image_index = 10 + k
    cfg = _cfg(densify_start_iter=10 ** 6, use_trained_exposure=True, exposure_lr_init=0.01,
               exposure_lr_final=0.001, exposure_max_iterations=100)
    tr = GaussianSplatTrainer(m, cams, gts, cfg, device=dev, seed=0, native=True)
    assert m.get_exposure.shape == (3, 3, 4) and m.image_id_to_index == {10: 0, 11: 1, 12: 2}
    for _ in range(6):
        tr.train_iteration()
    assert {lg.route for lg in tr.logs} == {"autograd"}
    sched = ExponentialLR(0.01, 0.001, max_steps=100)
    assert tr.exposure_optimizer.param_groups[0]["lr"] == pytest.approx(sched(6))
    eye = torch.eye(3, 4, device=dev)
    assert all(float((m.get_exposure[i] - eye).abs().max()) > 0 for i in range(3))
    assert bool(torch.isfinite(m.get_exposure).all())
    # coarse-to-fine: resolution 4, 2, 1 over thirds of min(20000, densify_end_iter)
    m2, cams2, gts2 = _problem(dev, n_true=20_000, n_init=4_000, W=320, H=240, views=2)
    tr2 = GaussianSplatTrainer(m2, cams2, gts2, _cfg(densify_start_iter=10 ** 6, densify_end_iter=30,
                                                     coarse_to_fine=True), device=dev, seed=0, native=True)
    seen = []
    for _ in range(32):
        tr2.train_iteration()
        seen.append(tr2.training_resolution())     # the iteration just run (train_iteration increments first)
    # threshold min(20000, 30) // 3 = 10: iterations 1-9 at 4, 10-19 at 2, then 1
    assert seen == [4] * 9 + [2] * 10 + [1] * 13
    assert [lg.route for lg in tr2.logs] == ["autograd"] * 19 + ["native"] * 13
    assert (tr2._scaled_views[(0, 4)][1].shape == (3, 60, 80)) and tr2._scaled_views[(0, 4)][0].width == 80
    assert bool(torch.isfinite(m2.get_xyz).all())
