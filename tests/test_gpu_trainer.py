"""The single-GPU training loop (dogs_amd.trainer.GaussianSplatTrainer: gaussian_trainer.py:324-513 inside
implicit_recon_trainer.py:296-353) and the model lifecycle it drives (dogs_amd.gaussian_model), on the GPU.

* The loop at BASELINE config 1's size (1e5-Gaussian synthetic scene, 800x800 targets rendered through the drop-in
  `_C` table), started from a 20k-point cloud (init_from_colmap_pcd: simple-knn scales, SH dc from the colours),
  with the reference's schedule shortened: densify every 100 iterations after 100 until 800, an opacity reset at
  500, a LightGaussian prune at 600, the SH degree raised every 250: 1000 iterations.  The events fire at the
  reference's iterations, the Gaussian count follows them, the PSNR against the targets rises by > 8 dB, and
  everything stays finite.
* The native route (dg_train_step per ordinary iteration, rebinding after every densify / reset / prune) and the
  autograd route (every iteration through render() + SparseGaussianAdam, as the reference's trainer calls the drop-in
  API) follow the same loss trajectory through three densifications (same split draws, same counts).
* A native step bound to tensors the model has since replaced refuses to run (no use-after-free); rebind() recovers.
* The device prune compaction (dg_prune_select + dg_densify_gather + dg_prune_gather_stats) equals torch's boolean
  indexing of every tensor, moment and statistic bit for bit; reset_opacity equals the reference's expression.
* A zero activated scale (exp underflow) gives the scale regulariser a finite gradient on both routes.
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cams(W, H, yaws, dev):
    from dogs_amd.camera import make_camera, yaw_world_to_camera
    return [make_camera(W, H, 1000.0, 1000.0, world_to_camera=yaw_world_to_camera(math.radians(y))).to(dev)
            for y in yaws]


@torch.no_grad()
def _render_raw(raw, cam, dev):
    from dogs_amd.diff_gaussian_rasterization import _C
    e = torch.empty(0, device=dev)
    out = _C.rasterize_gaussians(torch.zeros(3, device=dev), raw["xyz"], e, torch.sigmoid(raw["opacity"]),
                                 torch.exp(raw["scaling"]), torch.nn.functional.normalize(raw["quaternion"]), 1.0, e,
                                 cam.world_to_camera, cam.projective_matrix, cam.tanfovx, cam.tanfovy, cam.height,
                                 cam.width, raw["features_dc"], raw["features_rest"], 3, cam.camera_center, False,
                                 False, False)
    return out[2].clamp(0, 1).contiguous()


def _model_raw(m):
    return {"xyz": m._xyz.detach(), "features_dc": m._features_dc.detach(), "features_rest": m._features_rest.detach(),
            "opacity": m._opacity.detach(), "scaling": m._scaling.detach(), "quaternion": m._quaternion.detach()}


def _psnr(a, b):
    return -10.0 * math.log10(max(float(((a - b) ** 2).mean()), 1e-20))


def _problem(dev, n_true=100_000, n_init=20_000, W=800, H=800, views=8):
    from dogs_amd.gaussian_model import GaussianSplatModel
    from dogs_amd.synthetic import make_scene
    s = make_scene(n_true, W, H, fx=1000.0, fy=1000.0, seed=21)
    true = {"xyz": s.means3D.to(dev), "features_dc": s.dc.to(dev), "features_rest": s.sh.to(dev),
            "scaling": s.raw_scales.to(dev).contiguous(), "quaternion": s.raw_rotations.to(dev).contiguous(),
            "opacity": s.raw_opacities.to(dev).contiguous()}
    yaws = [0.0, 2.0, -2.0, 1.0, -1.0, 3.0, -3.0, 0.5][:views]
    cams = _cams(W, H, yaws, dev)
    gts = [_render_raw(true, c, dev) for c in cams]
    g = torch.Generator().manual_seed(5)
    pick = torch.randperm(n_true, generator=g)[:n_init]
    pts = s.means3D[pick].numpy()
    cols = (s.dc[pick, 0] * 0.28209479177387814 + 0.5).clamp(0, 1).numpy()
    m = GaussianSplatModel(3, 0.01, dev)
    m.init_from_colmap_pcd(pts, cols)
    return m, cams, gts


def _normal(dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    return lambda mean, std: torch.normal(mean, std, generator=g)


def _cfg(**kw):
    from dogs_amd.trainer import GSTrainConfig
    c = dict(max_iterations=1000, densify_start_iter=100, densify_end_iter=800, densification_interval=100,
             opacity_reset_interval=500, prune_iterations=(600,), sh_increase_interval=250, spatial_lr_scale=5.0)
    c.update(kw)
    return GSTrainConfig(**c)


def test_training_loop_schedule_and_learning(hip_device):
    from dogs_amd.trainer import GaussianSplatTrainer
    dev = hip_device
    m, cams, gts = _problem(dev)
    p0 = np.mean([_psnr(_render_raw(_model_raw(m), c, dev), g) for c, g in zip(cams, gts)])
    tr = GaussianSplatTrainer(m, cams, gts, _cfg(), device=dev, seed=0, native=True, normal=_normal(dev, 0))
    tr.train()
    assert tr.iteration == 1000
    ev = {lg.iteration: lg.events for lg in tr.logs if lg.events}
    assert sorted(i for i, e in ev.items() if "densify" in e) == [200, 300, 400, 500, 600, 700]
    assert [i for i, e in ev.items() if "reset_opacity" in e] == [500]
    assert [i for i, e in ev.items() if "prune" in e] == [600]
    assert sum(lg.route == "native" for lg in tr.logs) == 1000 - len(ev)
    counts = {lg.iteration: lg.num_gaussians for lg in tr.logs}
    raw = _model_raw(m)
    p1 = np.mean([_psnr(_render_raw(raw, c, dev), g) for c, g in zip(cams, gts)])
    print(f"PSNR {p0:.2f} -> {p1:.2f} dB; Gaussians per event {[(i, counts[i - 1], counts[i]) for i in sorted(ev)]}")
    # the count moves only at densify / prune iterations (clone + split - low-opacity prune; the prune's percentile)
    moved = sorted(i for i in range(2, 1001) if counts[i] != counts[i - 1])
    assert set(moved) <= {200, 300, 400, 500, 600, 700} and 600 in moved, moved
    assert counts[600] < counts[599]
    assert m.active_sh_degree == 3
    assert all(bool(torch.isfinite(t).all()) for t in raw.values())
    assert p1 > p0 + 8.0, (p0, p1)


def _route_state(tr):
    """Every tensor a training iteration writes: parameters, both Adam moments, the densification statistics."""
    tr.sync()
    m = tr.model
    out = {f"param.{k}": v.detach().clone() for k, v in m.params().items()}
    for g in tr.optimizer.param_groups:
        st = tr.optimizer.state[g["params"][0]]
        out[f"m.{g['name']}"], out[f"v.{g['name']}"] = st["exp_avg"].clone(), st["exp_avg_sq"].clone()
    out.update(grad_accum=m.xyz_gradient_accum.clone(), denom=m.denom.clone(), max_radii2D=m.max_radii2D.clone())
    return out


def _assert_same_state(a, b):
    for k in a:
        assert torch.equal(a[k], b[k]), (k, float((a[k].double() - b[k].double()).abs().max()))


def test_native_and_autograd_routes_agree_through_densify(hip_device):
    """The native route (dg_train_step) and the autograd route (render() + fused_ssim + row_prod + SparseGaussianAdam,
    the reference trainer's calls) run the same kernels, and the native step forms every loss gradient as torch's
    autograd forms it (mean backward as a multiply by the float reciprocal, the activations' and the masked L1's
    association), so the two trajectories are bit-identical through three densifications: the same
    Gaussian counts at every iteration and bitwise-equal parameters, Adam moments and statistics at the end.  Only the
    logged loss differs, by rounding (its value is summed in a different order on each route)."""
    from dogs_amd.trainer import GaussianSplatTrainer
    dev = hip_device
    cfg = _cfg(max_iterations=200, densify_start_iter=20, densification_interval=40, prune_iterations=(),
               opacity_reset_interval=10 ** 6, sh_increase_interval=60)
    runs = []
    for native in (True, False):
        m, cams, gts = _problem(dev, n_true=30_000, n_init=6_000, W=400, H=400, views=4)
        tr = GaussianSplatTrainer(m, cams, gts, cfg, device=dev, seed=1, native=native, normal=_normal(dev, 7))
        losses, counts = [], []
        for _ in range(130):
            tr.train_iteration()
            losses.append(float(tr.loss()))
            counts.append(m.num_gaussians)
        runs.append((np.array(losses), np.array(counts), [lg.route for lg in tr.logs], _route_state(tr)))
    (l0, c0, r0, s0), (l1, c1, r1, s1) = runs
    assert r0.count("autograd") == 3 and set(r1) == {"autograd"}      # densify at 40, 80, 120
    print("counts", c0[[38, 39, 78, 79, 118, 119]], "max rel loss diff", float(np.max(np.abs(l0 - l1) / l1)))
    assert c0[38] == 6000 and c0[39] != 6000                            # index i = iteration i + 1: densify at 40
    np.testing.assert_array_equal(c0, c1)
    _assert_same_state(s0, s1)
    np.testing.assert_allclose(l0, l1, rtol=1e-5)


def test_stale_native_binding_refused(hip_device):
    from dogs_amd.trainer import GaussianSplatTrainer
    dev = hip_device
    m, cams, gts = _problem(dev, n_true=20_000, n_init=4_000, W=320, H=240, views=2)
    tr = GaussianSplatTrainer(m, cams, gts, _cfg(densify_start_iter=10 ** 6), device=dev, seed=0, native=True)
    tr.train_iteration()
    nts = tr._nts
    m.reset_opacity(tr.optimizer)                    # replaces the opacity tensor and its moments
    with pytest.raises(RuntimeError, match="rebind"):
        nts.step(0, 1e-4)
    tr._rebind()
    nts.step(0, 1e-4)
    torch.cuda.synchronize()


def test_prune_compaction_matches_torch(hip_device):
    from dogs_amd.diff_gaussian_rasterization import SparseGaussianAdam
    from dogs_amd.gaussian_model import GaussianSplatModel
    dev = hip_device
    g = torch.Generator().manual_seed(3)
    for n, degree in ((50_001, 3), (777, 1), (1, 3)):
        M = (degree + 1) ** 2 - 1
        m = GaussianSplatModel(degree, 0.01, dev)
        m.init_from_external_properties(*(torch.randn(s, generator=g) for s in
                                          ((n, 3), (n, 1, 3), (n, M, 3), (n, 3), (n, 4), (n, 1))), optimizable=True)
        m.xyz_gradient_accum = torch.rand((n, 1), generator=g).to(dev)
        m.denom = torch.rand((n, 1), generator=g).to(dev)
        m.max_radii2D = torch.rand((n,), generator=g).to(dev)
        opt = SparseGaussianAdam([{"params": [p], "lr": 0.1, "name": k} for k, p in m.params().items()], 0.0, 1e-15)
        for p in m.params().values():
            opt.state[p] = {"step": torch.tensor(0.0), "exp_avg": torch.randn(p.shape, generator=g).to(dev),
                            "exp_avg_sq": torch.rand(p.shape, generator=g).to(dev)}
        mask = (torch.rand(n, generator=g) < 0.37).to(dev)
        keep = ~mask
        want = {k: (p.detach()[keep], opt.state[p]["exp_avg"][keep], opt.state[p]["exp_avg_sq"][keep])
                for k, p in m.params().items()}
        wstats = (m.xyz_gradient_accum[keep], m.denom[keep], m.max_radii2D[keep])
        n_out = m.prune_points(mask, opt)
        assert n_out == int(keep.sum())
        for k, p in m.params().items():
            assert opt.param_groups[[gg["name"] for gg in opt.param_groups].index(k)]["params"][0] is p
            assert isinstance(p, torch.nn.Parameter) and p.requires_grad
            assert torch.equal(p.detach(), want[k][0])
            assert torch.equal(opt.state[p]["exp_avg"], want[k][1])
            assert torch.equal(opt.state[p]["exp_avg_sq"], want[k][2])
        for a, b in zip((m.xyz_gradient_accum, m.denom, m.max_radii2D), wstats):
            assert torch.equal(a, b)


def test_reset_opacity_and_percentile(hip_device):
    from dogs_amd.diff_gaussian_rasterization import SparseGaussianAdam
    from dogs_amd.gaussian_model import GaussianSplatModel, inverse_sigmoid
    dev = hip_device
    g = torch.Generator().manual_seed(4)
    n = 10_000
    m = GaussianSplatModel(3, 0.01, dev)
    m.init_from_external_properties(*(torch.randn(s, generator=g) * 3 for s in
                                      ((n, 3), (n, 1, 3), (n, 15, 3), (n, 3), (n, 4), (n, 1))), optimizable=True)
    opt = SparseGaussianAdam([{"params": [p], "lr": 0.1, "name": k} for k, p in m.params().items()], 0.0, 1e-15)
    for p in m.params().values():
        opt.state[p] = {"step": torch.tensor(0.0), "exp_avg": torch.ones_like(p), "exp_avg_sq": torch.ones_like(p)}
    want = inverse_sigmoid(torch.min(torch.sigmoid(m._opacity.detach()), torch.ones_like(m._opacity) * 0.01))
    m.reset_opacity(opt)
    assert torch.equal(m._opacity.detach(), want)
    assert float(opt.state[m._opacity]["exp_avg"].abs().max()) == 0.0
    assert opt.param_groups[3]["params"][0] is m._opacity
    score = torch.rand(n, generator=g).to(dev)
    s, _ = torch.sort(score)
    thr = s[int(0.3 * (n - 1))]
    n_out = m.prune_gaussians_with_opt(0.3, score, opt)
    assert n_out == int((score > thr).sum())


def test_underflowed_scale_has_finite_regulariser_gradient(hip_device):
    """exp(raw scale) == 0 for very negative raw scales: the scale regulariser's gradient is the product of the other
    two columns (torch's prod backward on zeros), finite on the native route and equal to the autograd route's."""
    from dogs_amd.admm import ADMMConfig
    from dogs_amd.admm_trainer import BlockTrainer, TrainConfig
    from dogs_amd.synthetic import make_scene
    dev = hip_device
    s = make_scene(5_000, 320, 240, seed=9)
    raw = {"xyz": s.means3D, "features_dc": s.dc, "features_rest": s.sh, "scaling": s.raw_scales.clone(),
           "quaternion": s.raw_rotations, "opacity": s.raw_opacities}
    raw["scaling"][:50, 1] = -200.0                  # exp underflows to exactly 0
    cams = _cams(320, 240, [0.0, 1.0], dev)
    gts = [torch.rand(3, 240, 320, generator=torch.Generator().manual_seed(k)).to(dev) for k in range(2)]
    off = ADMMConfig(alpha_xyz=0.0, alpha_fdc=0.0, alpha_fr=0.0, alpha_s=0.0, alpha_q=0.0, alpha_o=0.0)
    cfg = TrainConfig(lambda_scale=10.0)
    trs = [BlockTrainer(raw, cams, gts, 5_000, off, cfg, dev, seed=0, native=nat) for nat in (True, False)]
    for _ in range(3):
        for t in trs:
            t.local_step()
    a, b = (t.params["scaling"].detach() for t in trs)
    assert bool(torch.isfinite(a).all()) and bool(torch.isfinite(b).all())
    torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_overlapped_update_is_bitwise_the_serial_one(hip_device):
    """GaussianSplatTrainer(overlap=True) -- each native step's f_dc / f_rest update on a side stream beside the next
    step's forward -- ends with the same model, Adam state and statistics bit for bit as overlap=False, through a
    densification and an opacity reset (autograd-route iterations in between sync first)."""
    from dogs_amd.trainer import GaussianSplatTrainer
    dev = hip_device
    cfg = _cfg(max_iterations=90, densify_start_iter=30, densification_interval=40, opacity_reset_interval=60,
               prune_iterations=(), sh_increase_interval=25)
    out = []
    for overlap in (False, True):
        m, cams, gts = _problem(dev, n_true=20_000, n_init=4_000, W=320, H=240, views=4)
        tr = GaussianSplatTrainer(m, cams, gts, cfg, device=dev, seed=3, native=True, normal=_normal(dev, 11),
                                  overlap=overlap)
        tr.train()
        assert tr._nts.overlap == overlap
        opt = {g["name"]: tr.optimizer.state[g["params"][0]] for g in tr.optimizer.param_groups}
        out.append((_model_raw(m), {k: (v["exp_avg"].clone(), v["exp_avg_sq"].clone()) for k, v in opt.items()},
                    (m.max_radii2D.clone(), m.xyz_gradient_accum.clone(), m.denom.clone()),
                    [lg.route for lg in tr.logs]))
    (r0, o0, s0, l0), (r1, o1, s1, l1) = out
    assert l0 == l1 and l0.count("autograd") >= 2
    for k in r0:
        assert torch.equal(r0[k], r1[k]), k
    for k in o0:
        assert torch.equal(o0[k][0], o1[k][0]) and torch.equal(o0[k][1], o1[k][1]), k
    for a, b in zip(s0, s1):
        assert torch.equal(a, b)


def test_training_loop_1080p(hip_device):
    """BASELINE config 2's image size: 1920 x 1080 targets of a 1e6-Gaussian scene, the loop from a 100k-point cloud for
    300 iterations (densify at 100 and 200, an opacity reset at 150, statistics on throughout): the schedule, the
    count changes at the densifications only, the PSNR rises, everything finite."""
    from dogs_amd.trainer import GaussianSplatTrainer
    dev = hip_device
    m, cams, gts = _problem(dev, n_true=1_000_000, n_init=100_000, W=1920, H=1080, views=8)
    p0 = np.mean([_psnr(_render_raw(_model_raw(m), c, dev), g) for c, g in zip(cams, gts)])
    cfg = _cfg(max_iterations=300, densify_start_iter=50, densify_end_iter=300, densification_interval=100,
               opacity_reset_interval=150, prune_iterations=(), sh_increase_interval=100)
    tr = GaussianSplatTrainer(m, cams, gts, cfg, device=dev, seed=0, native=True, normal=_normal(dev, 2))
    tr.train()
    ev = {lg.iteration: lg.events for lg in tr.logs if lg.events}
    assert ev == {100: ["densify"], 150: ["reset_opacity"], 200: ["densify"]}, ev
    counts = {lg.iteration: lg.num_gaussians for lg in tr.logs}
    moved = sorted(i for i in range(2, 301) if counts[i] != counts[i - 1])
    assert moved == [100, 200], moved
    raw = _model_raw(m)
    p1 = np.mean([_psnr(_render_raw(raw, c, dev), g) for c, g in zip(cams, gts)])
    print(f"1080p PSNR {p0:.2f} -> {p1:.2f} dB; Gaussians {counts[1]} -> {counts[300]}")
    assert all(bool(torch.isfinite(t).all()) for t in raw.values())
    assert p1 > p0 + 3.0, (p0, p1)


def test_native_and_autograd_routes_agree_1080p(hip_device):
    """At 1920 x 1080 through a densification: the two routes are bit-identical (counts at every iteration, the
    final parameters, moments and statistics), the logged losses equal to rounding."""
    from dogs_amd.trainer import GaussianSplatTrainer
    dev = hip_device
    cfg = _cfg(max_iterations=120, densify_start_iter=20, densify_end_iter=110, densification_interval=50,
               prune_iterations=(), opacity_reset_interval=10 ** 6, sh_increase_interval=40)
    runs = []
    for native in (True, False):
        m, cams, gts = _problem(dev, n_true=300_000, n_init=40_000, W=1920, H=1080, views=4)
        tr = GaussianSplatTrainer(m, cams, gts, cfg, device=dev, seed=1, native=native, normal=_normal(dev, 7))
        losses, counts = [], []
        for _ in range(70):
            tr.train_iteration()
            losses.append(float(tr.loss()))
            counts.append(m.num_gaussians)
        runs.append((np.array(losses), np.array(counts), _route_state(tr)))
    (l0, c0, s0), (l1, c1, s1) = runs
    print("1080p max rel loss diff", float(np.max(np.abs(l0 - l1) / l1)), "counts after", c0[49], c1[49])
    assert c0[48] == 40_000 and c0[49] != 40_000
    np.testing.assert_array_equal(c0, c1)
    _assert_same_state(s0, s1)
    np.testing.assert_allclose(l0, l1, rtol=1e-5)


def test_overlap_with_two_view_sizes_is_bitwise_serial(hip_device):
    """Views of two image sizes alternate (the step's scratch block is handed back for either size): the overlapped
    f_dc / f_rest update reads its gradients from an offset that does not depend on the image size, so overlap=True
    ends bit-identical to overlap=False (the gradients used to follow the image-sized buffers)."""
    from dogs_amd.camera import make_camera, yaw_world_to_camera
    from dogs_amd.trainer import GaussianSplatTrainer
    dev = hip_device
    cfg = _cfg(max_iterations=24, densify_start_iter=10 ** 6, opacity_reset_interval=10 ** 6, prune_iterations=(),
               sh_increase_interval=6)
    out = []
    for overlap in (False, True):
        m, _, _ = _problem(dev, n_true=20_000, n_init=4_000, W=320, H=240, views=1)
        cams = [make_camera(w, h, 500.0, 500.0, world_to_camera=yaw_world_to_camera(math.radians(y))).to(dev)
                for (w, h), y in (((320, 240), 0.0), ((512, 384), 1.0), ((320, 240), -1.0), ((512, 384), 2.0))]
        g = torch.Generator().manual_seed(3)
        gts = [torch.rand((3, c.height, c.width), generator=g).to(dev) for c in cams]
        tr = GaussianSplatTrainer(m, cams, gts, cfg, device=dev, seed=5, native=True, overlap=overlap)
        tr.train()
        assert {lg.route for lg in tr.logs} == {"native"}
        out.append((_model_raw(m), {g_["name"]: tr.optimizer.state[g_["params"][0]]["exp_avg"].clone()
                                    for g_ in tr.optimizer.param_groups}))
    for k in out[0][0]:
        assert torch.equal(out[0][0][k], out[1][0][k]), k
    for k in out[0][1]:
        assert torch.equal(out[0][1][k], out[1][1][k]), k


def test_capacity_context_released_with_trainer(hip_device):
    """a trainer's own adaptive-capacity context (its device probe and state in the library) is released
    when the trainer is garbage collected; dg_adaptive_capacity(reset) resets every context of the image size and
    dg_adaptive_capacity_ctx queries one."""
    import gc
    from dogs_amd import _lib
    from dogs_amd.trainer import GaussianSplatTrainer
    gc.collect()
    torch.cuda.synchronize()
    n0 = _lib.capacity_contexts()
    m, cams, gts = _problem(hip_device, n_true=20_000, n_init=4_000, W=320, H=240, views=2)
    tr = GaussianSplatTrainer(m, cams, gts, _cfg(densify_start_iter=10 ** 6), device=hip_device, seed=0, native=True)
    for _ in range(3):
        tr.train_iteration()
    tr.sync()
    torch.cuda.synchronize()
    ctx = tr.capacity_ctx
    assert _lib.capacity_contexts() == n0 + 1
    _lib.adaptive_capacity(320, 240, reset=True)
    assert _lib.adaptive_capacity_ctx(ctx, 320, 240) == _lib.adaptive_capacity(320, 240)
    del tr
    gc.collect()
    torch.cuda.synchronize()
    assert _lib.capacity_contexts() == n0
