"""GPU parity of the auxiliary ops against the CPU oracle (all through the drop-in Python surface, i.e. the
C-ABI library): fused-SSIM forward/backward (ssim.cu:187-444), sparse Adam (adam.cu:10-38), simple-knn distCUDA2
(simple_knn.cu:45-221), markVisible / filter radii (rasterize_points.cu:254-334), and the autograd wrapper
GaussianRasterizer (dc/sh split, depth_threshold scaling) end to end.

Bars: integer/index work and correctly-rounded fp32 elementwise code bit-exact; SSIM: the kernel sums the window in
another float32 order than ssim.cu (Horner form), so each map's error against the float64 value
(oracle.ssim_forward_exact) is held to twice the reference order's own float32 error, and every array is within 1e-5
norm-wise relative error, and 3e-5 of the array's scale element by element, of the C restatement.  The largest
cases are the BASELINE sizes: SSIM at 1 x 3 x 1080 x 1920, distCUDA2 at 1e6 points (tests/test_gpu_optim.py runs
SparseGaussianAdam at 1e6 x 59)."""
import numpy as np
import pytest
import torch

from raster_util import oracle_forward, rel_err, small_scene

pytestmark = pytest.mark.gpu


def _within_reference_order_error(x, ref32, exact, name):
    """The GPU kernel sums the 11-tap window in another float32 order than ssim.cu (Horner form over the lanes,
    aux_kernels.hip hconv11) and takes reciprocals instead of IEEE divisions.  Bar: its error against the float64 value
    is at most twice the reference order's own float32 error (the C restatement, which sums in ssim.cu's order)
    plus 1e-6 of the array's scale.  Measured by a float32 emulation of both orders: ratio 0.7-1.4 over these shapes."""
    x = np.asarray(x, np.float64)
    e_ref = float(np.abs(np.asarray(ref32, np.float64) - exact).max())
    e_ours = float(np.abs(x - exact).max())
    scale = max(1.0, float(np.abs(exact).max()))
    assert e_ours <= 2.0 * e_ref + 1e-6 * scale, (name, e_ours, e_ref, scale)
    assert rel_err(x, ref32) < 1e-5, name
    # and element by element against the restatement (round 4's Horner change measured 2.4e-5 at worst), so that a
    # regression confined to a few pixels cannot hide inside the norm
    d = float(np.abs(x - np.asarray(ref32, np.float64)).max())
    assert d <= 3e-5 * scale, (name, d, scale)


# several strips across (54 output columns per wave) with even and odd widths, ragged rows (32 per strip)
@pytest.mark.parametrize("B,C,H,W", [(1, 3, 37, 53), (1, 3, 128, 96), (2, 1, 64, 64), (1, 3, 70, 250),
                                     (1, 1, 33, 237), (1, 2, 5, 119), (1, 3, 1080, 1920)])
def test_fused_ssim_matches_oracle(oracle, hip_device, B, C, H, W):
    from fused_ssim_cuda import fusedssim, fusedssim_backward
    g = torch.Generator().manual_seed(H * W)
    a = torch.rand((B, C, H, W), generator=g)
    b = (a + 0.1 * torch.randn((B, C, H, W), generator=g)).clamp(0, 1)
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    ref = oracle.ssim_forward(a.numpy(), b.numpy(), C1, C2)
    exact = oracle.ssim_forward_exact(a.numpy(), b.numpy(), C1, C2)
    got = fusedssim(C1, C2, a.to(hip_device), b.to(hip_device), True)
    for x, r, e, nm in zip(got, ref, exact, ("map", "dm_dmu1", "dm_dsigma1_sq", "dm_dsigma12")):
        _within_reference_order_error(x.cpu().numpy(), r, e, nm)
    dmap = torch.randn((B, C, H, W), generator=g)
    d1_o, d2_o, d3_o = ref[1:]
    go = oracle.ssim_backward(a.numpy(), b.numpy(), dmap.numpy(), d1_o, d2_o, d3_o)
    # the backward kernel alone, on the oracle's maps
    gh = fusedssim_backward(C1, C2, a.to(hip_device), b.to(hip_device), dmap.to(hip_device),
                            *[torch.from_numpy(d).to(hip_device) for d in (d1_o, d2_o, d3_o)])
    _within_reference_order_error(gh.cpu().numpy(), go, oracle.ssim_backward_exact(a.numpy(), b.numpy(),
                                                                                      dmap.numpy(), d1_o, d2_o, d3_o),
                                  "dL_dimg1")
    # end to end, on the GPU's own maps
    gh = fusedssim_backward(C1, C2, a.to(hip_device), b.to(hip_device), dmap.to(hip_device), *got[1:])
    assert rel_err(gh.cpu().numpy(), go) < 1e-5


@pytest.mark.parametrize("B,C,H,W", [(1, 3, 37, 53), (2, 1, 64, 64), (1, 2, 5, 119), (1, 3, 1080, 1920)])
def test_fused_ssim_mean_matches_map_route(hip_device, B, C, H, W):
    """fused_ssim(padding="same") runs FusedSSIMMean (the map's mean summed in the kernel, the backward from the mean's
    scalar gradient): its value equals FusedSSIMMap(...).mean() to float association (a fixed-order sum of per-wave
    partials vs torch's mean), its gradient equals the map route's bit for bit (dL/dmap = g / numel either way), and
    train=False gives the same value without the partial maps."""
    from fused_ssim import FusedSSIMMap, fused_ssim
    g = torch.Generator().manual_seed(H + W)
    a = torch.rand((B, C, H, W), generator=g).to(hip_device)
    b = (a.cpu() + 0.1 * torch.randn((B, C, H, W), generator=g)).clamp(0, 1).to(hip_device)
    x1, x2 = a.clone().requires_grad_(True), a.clone().requires_grad_(True)
    v = fused_ssim(x1, b)
    m = FusedSSIMMap.apply(0.01 ** 2, 0.03 ** 2, x2, b, "same", True).mean()
    assert v.dim() == 0 and v.dtype == torch.float32
    assert abs(v.item() - m.item()) <= 2e-6 * abs(m.item()) + 1e-7, (v.item(), m.item())
    (-0.2 * v).backward()
    (-0.2 * m).backward()
    assert torch.equal(x1.grad, x2.grad)
    assert torch.equal(fused_ssim(a, b, train=False), v.detach())


def test_fused_ssim_autograd_valid_padding(oracle, hip_device):
    from fused_ssim import fused_ssim
    g = torch.Generator().manual_seed(3)
    a = torch.rand((1, 3, 40, 44), generator=g)
    b = torch.rand((1, 3, 40, 44), generator=g)
    x = a.to(hip_device).requires_grad_(True)
    v = fused_ssim(x, b.to(hip_device), padding="valid")
    v.backward()
    mp_o, d1, d2, d3 = oracle.ssim_forward(a.numpy(), b.numpy())
    ref = float(mp_o[:, :, 5:-5, 5:-5].mean(dtype=np.float64))
    assert abs(v.item() - ref) < 1e-5
    dmap = np.zeros_like(mp_o)
    dmap[:, :, 5:-5, 5:-5] = 1.0 / mp_o[:, :, 5:-5, 5:-5].size
    go = oracle.ssim_backward(a.numpy(), b.numpy(), dmap, d1, d2, d3)
    assert rel_err(x.grad.cpu().numpy(), go) < 1e-5


@pytest.mark.parametrize("N,M", [(1000, 3), (777, 45), (64, 1)])
def test_sparse_adam_bitexact(oracle, hip_device, N, M):
    from diff_gaussian_rasterization import _C
    g = torch.Generator().manual_seed(N + M)
    p, gr = torch.randn((N, M), generator=g), torch.randn((N, M), generator=g)
    m, v = torch.randn((N, M), generator=g), torch.rand((N, M), generator=g)
    vis = torch.rand(N, generator=g) > 0.3
    po, mo, vo = p.numpy().copy(), m.numpy().copy(), v.numpy().copy()
    oracle.adam(po, gr.numpy().copy(), mo, vo, vis.numpy(), 1e-3, 0.9, 0.999, 1e-15, N, M)
    ph, mh, vh = p.to(hip_device), m.to(hip_device), v.to(hip_device)
    _C.adamUpdate(ph, gr.to(hip_device), mh, vh, vis.to(hip_device), 1e-3, 0.9, 0.999, 1e-15, N, M)
    np.testing.assert_array_equal(ph.cpu().numpy(), po)
    np.testing.assert_array_equal(mh.cpu().numpy(), mo)
    np.testing.assert_array_equal(vh.cpu().numpy(), vo)


@pytest.mark.parametrize("P", [1, 5, 1000, 20000, 1_000_000])
def test_dist_cuda2_bitexact(oracle, hip_device, P):
    from simple_knn._C import distCUDA2
    g = torch.Generator().manual_seed(P)
    pts = torch.randn((P, 3), generator=g) * torch.tensor([3.0, 1.0, 0.5])
    ref = oracle.knn_dist2(pts.numpy())
    got = distCUDA2(pts.to(hip_device)).cpu().numpy()
    np.testing.assert_array_equal(got, ref)


def test_mark_visible_and_filter_bitexact(oracle, hip_device):
    from diff_gaussian_rasterization import _C
    s = small_scene(3000, 200, 150, seed=9)
    s.means3D[:100, 2] = -1.0              # behind the camera
    c = s.camera
    vis_o = oracle.mark_visible(s.means3D.numpy(), c.world_to_camera.numpy(), c.projective_matrix.numpy())
    vis = _C.mark_visible(s.means3D.to(hip_device), c.world_to_camera.to(hip_device), c.projective_matrix.to(hip_device))
    np.testing.assert_array_equal(vis.cpu().numpy(), vis_o)
    r_o = oracle.filter_radii(s.means3D.numpy(), c.world_to_camera.numpy(), c.projective_matrix.numpy(), c.tanfovx,
                              c.tanfovy, 150, 200, scales=s.scales.numpy(), rotations=s.rotations.numpy())
    e = torch.empty(0, device=hip_device)
    d = lambda t: t.to(hip_device).contiguous()  # noqa: E731
    r = _C.rasterize_gaussians_filter(d(s.means3D), d(s.scales), d(s.rotations), 1.0, e, d(c.world_to_camera),
                                      d(c.projective_matrix), c.tanfovx, c.tanfovy, 150, 200, False, False)
    np.testing.assert_array_equal(r.cpu().numpy(), r_o)


def test_several_grad_forwards_hold_one_plan(hip_device):
    """the autograd forward prepares its backward's buffers ahead (BackwardPlan) only while no other plan on
    the device holds them.  Two grad-mode renders before one backward: the second allocates nothing ahead (its
    forward grows the allocated memory by less than the first one's plan), both backwards give the gradients of
    separate single-view backwards bit for bit, and every slot is handed back -- after the backwards, and when a
    grad-mode render is dropped without a backward."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from dogs_amd.diff_gaussian_rasterization import _C
    n, W, H = 200_000, 1280, 720
    s = small_scene(n, W, H, seed=33)
    c = s.camera.to(hip_device)
    st = GaussianRasterizationSettings(image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy,
                                       bg=torch.zeros(3, device=hip_device), scale_modifier=1.0,
                                       viewmatrix=c.world_to_camera, projmatrix=c.projective_matrix, sh_degree=3,
                                       campos=c.camera_center, prefiltered=False, debug=False)
    r = GaussianRasterizer(st)
    leaf = {k: getattr(s, k).to(hip_device).clone().requires_grad_(True)
            for k in ("means3D", "opacities", "scales", "rotations", "dc", "sh")}
    g1 = torch.randn((3, H, W), generator=torch.Generator().manual_seed(1)).to(hip_device)
    g2 = torch.randn((3, H, W), generator=torch.Generator().manual_seed(2)).to(hip_device)

    def render():
        m2 = torch.zeros_like(leaf["means3D"], requires_grad=True)
        return r(leaf["means3D"], m2, leaf["opacities"], dc=leaf["dc"], shs=leaf["sh"], scales=leaf["scales"],
                 rotations=leaf["rotations"])[0]

    def grads():
        out = {k: t.grad.clone() for k, t in leaf.items()}
        for t in leaf.values():
            t.grad = None
        return out

    old = _C.set_prefix_per_tile(448)     # a fixed phase-1 capacity: the same instance numbering in every render
    try:
        _two_forwards_one_backward(render, grads, leaf, g1, g2, n, hip_device)
    finally:
        _C.set_prefix_per_tile(old)


def _two_forwards_one_backward(render, grads, leaf, g1, g2, n, hip_device):
    from dogs_amd.diff_gaussian_rasterization import _C
    torch.cuda.synchronize()
    assert _C.eager_plans(hip_device) == 0
    (render() * g1).sum().backward()
    want1 = grads()
    (render() * g2).sum().backward()
    want2 = grads()
    assert _C.eager_plans(hip_device) == 0
    torch.cuda.synchronize()
    m0 = torch.cuda.memory_allocated(hip_device)
    a = render()
    torch.cuda.synchronize()
    m1 = torch.cuda.memory_allocated(hip_device)
    b = render()
    torch.cuda.synchronize()
    m2 = torch.cuda.memory_allocated(hip_device)
    assert _C.eager_plans(hip_device) == 1
    plan_bytes = n * (3 + 3 + 1 + 3 + 6 + 3 + 45 + 3 + 4 + 1) * 4
    assert (m2 - m1) < (m1 - m0) - plan_bytes // 2, (m0, m1, m2, plan_bytes)
    (a * g1).sum().backward()
    got1 = grads()
    (b * g2).sum().backward()
    got2 = grads()
    assert _C.eager_plans(hip_device) == 0
    for k in leaf:
        assert torch.equal(got1[k], want1[k]), k
        assert torch.equal(got2[k], want2[k]), k
    d = render()            # a grad-mode render kept for a metric, then dropped without a backward
    assert _C.eager_plans(hip_device) == 1
    del d
    assert _C.eager_plans(hip_device) == 0


def test_gaussian_rasterizer_autograd(oracle, hip_device):
    """GaussianRasterizer (the import surface callers use) end to end: forward image and the autograd gradients
    of means3D / dc / sh / opacities / scales / rotations against the oracle, depth_threshold = 0."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    n, W, H = 1500, 160, 120
    s = small_scene(n, W, H, seed=31)
    c = s.camera.to(hip_device)
    bg = torch.tensor([0.2, 0.1, 0.0], device=hip_device)
    st = GaussianRasterizationSettings(image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, bg=bg,
                                       scale_modifier=1.0, viewmatrix=c.world_to_camera,
                                       projmatrix=c.projective_matrix, sh_degree=3, campos=c.camera_center,
                                       prefiltered=False, debug=False, antialiasing=False, depth_threshold=0.0)
    r = GaussianRasterizer(st)
    leaf = {k: getattr(s, k).to(hip_device).clone().requires_grad_(True)
            for k in ("means3D", "opacities", "scales", "rotations", "dc", "sh")}
    means2D = torch.zeros_like(leaf["means3D"], requires_grad=True)
    img, radii, invd = r(leaf["means3D"], means2D, leaf["opacities"], dc=leaf["dc"], shs=leaf["sh"],
                         scales=leaf["scales"], rotations=leaf["rotations"])
    col_o, radii_o, inv_o, sto = oracle_forward(oracle, s, bg.cpu().numpy())
    np.testing.assert_array_equal(radii.cpu().numpy(), radii_o)
    assert np.abs(img.detach().cpu().numpy() - col_o).max() < 5e-3
    gen = np.random.default_rng(1)
    gc = gen.standard_normal((3, H, W)).astype(np.float32)
    (img * torch.from_numpy(gc).to(hip_device)).sum().backward()
    go = sto.backward(gc, np.zeros((H, W), np.float32))
    pairs = {"means3D": "dmeans3D", "opacities": "dopacity", "scales": "dscales", "rotations": "drot",
             "dc": "ddc", "sh": "dsh"}
    for k, o in pairs.items():
        assert rel_err(leaf[k].grad.cpu().numpy().reshape(go[o].shape), go[o]) < 1e-4, k
    assert rel_err(means2D.grad.cpu().numpy(), go["dmeans2D"]) < 1e-4
    # only the inverse depth in the loss: the image's gradient arrives as None (set_materialize_grads(False)) and
    # counts as zeros; and the image alone again, the inverse depth's gradient None -> NULL to the library
    ginv = (0.1 * gen.standard_normal((1, H, W))).astype(np.float32)
    for use_img, use_inv in ((False, True), (True, False)):
        for t in leaf.values():
            t.grad = None
        means2D = torch.zeros_like(leaf["means3D"], requires_grad=True)
        img, radii, invd = r(leaf["means3D"], means2D, leaf["opacities"], dc=leaf["dc"], shs=leaf["sh"],
                             scales=leaf["scales"], rotations=leaf["rotations"])
        loss = (invd * torch.from_numpy(ginv).to(hip_device)).sum() if use_inv else \
            (img * torch.from_numpy(gc).to(hip_device)).sum()
        loss.backward()
        go = sto.backward(gc if use_img else np.zeros_like(gc), ginv[0] if use_inv else np.zeros((H, W), np.float32))
        for k, o in pairs.items():
            assert rel_err(leaf[k].grad.cpu().numpy().reshape(go[o].shape), go[o]) < 1e-4, (k, use_img)
        assert rel_err(means2D.grad.cpu().numpy(), go["dmeans2D"]) < 1e-4


def test_planned_backward_equals_direct_call(hip_device):
    """_RasterizeGaussians prepares its backward during the forward (_C.backward_plan: outputs, argument struct and the
    DG_BUF_BACKWARD scratch through dg_fixed_alloc); its gradients equal the direct _C.rasterize_gaussians_backward
    call's bit for bit, with and without an inverse-depth gradient (each forward under a fresh capacity context, so both
    bin with the same phase-1 capacity), and a no_grad forward renders the same image."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from dogs_amd.diff_gaussian_rasterization import _C
    n, W, H = 3000, 200, 150
    s = small_scene(n, W, H, seed=41)
    c = s.camera.to(hip_device)
    bg = torch.tensor([0.0, 0.0, 0.0], device=hip_device)
    st = GaussianRasterizationSettings(image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, bg=bg,
                                       scale_modifier=1.0, viewmatrix=c.world_to_camera,
                                       projmatrix=c.projective_matrix, sh_degree=3, campos=c.camera_center,
                                       prefiltered=False, debug=False, antialiasing=False, depth_threshold=0.0)
    r = GaussianRasterizer(st)
    gen = torch.Generator().manual_seed(2)
    gc = torch.randn((3, H, W), generator=gen).to(hip_device)
    gi = (0.1 * torch.randn((1, H, W), generator=gen)).to(hip_device)
    d = {k: getattr(s, k).to(hip_device).contiguous() for k in ("means3D", "opacities", "scales", "rotations", "dc", "sh")}
    e = torch.empty(0, device=hip_device)
    for use_inv in (False, True):
        leaf = {k: v.clone().requires_grad_(True) for k, v in d.items()}
        m2d = torch.zeros_like(leaf["means3D"], requires_grad=True)
        with _C.capacity_context(_C.new_capacity_context()):
            img, radii, invd = r(leaf["means3D"], m2d, leaf["opacities"], dc=leaf["dc"], shs=leaf["sh"],
                                 scales=leaf["scales"], rotations=leaf["rotations"])
        loss = (img * gc).sum() + ((invd * gi).sum() if use_inv else 0.0)
        loss.backward()
        with _C.capacity_context(_C.new_capacity_context()):
            out = _C.rasterize_gaussians(bg, d["means3D"], e, d["opacities"], d["scales"], d["rotations"], 1.0, e,
                                         c.world_to_camera, c.projective_matrix, c.tanfovx, c.tanfovy, H, W, d["dc"],
                                         d["sh"], 3, c.camera_center, False, False, False)
        g = _C.rasterize_gaussians_backward(bg, d["means3D"], out[4], e, d["opacities"], d["scales"], d["rotations"],
                                            1.0, e, c.world_to_camera, c.projective_matrix, c.tanfovx, c.tanfovy, gc,
                                            d["dc"], d["sh"], gi if use_inv else None, 3, c.camera_center, out[5],
                                            out[0], out[6], out[7], out[1], out[8], False, False)
        torch.cuda.synchronize()
        assert torch.equal(m2d.grad, g[0])
        for k, gk in (("opacities", g[2]), ("means3D", g[3]), ("dc", g[5]), ("sh", g[6]), ("scales", g[7]),
                      ("rotations", g[8])):
            assert torch.equal(leaf[k].grad, gk.reshape(leaf[k].shape)), (k, use_inv)
    with torch.no_grad(), _C.capacity_context(_C.new_capacity_context()):
        img2, _, _ = r(d["means3D"], torch.zeros_like(d["means3D"]), d["opacities"], dc=d["dc"], shs=d["sh"],
                       scales=d["scales"], rotations=d["rotations"])
    assert torch.equal(img2, img.detach())


@pytest.mark.parametrize("prefix", [0, 2], ids=["prefix-default", "prefix-2-per-tile"])
def test_count_mode_matches_oracle(oracle, hip_device, prefix):
    """LightGaussian count mode (GaussianRasterizationSettings(f_count=True), as count_render,
    conerf/render/gaussian_render.py:161-278, calls it with the full SH features): per-Gaussian contributing-pixel
    counts and importance scores against the oracle's restatement of renderCUDA_count (old forward.cu:392-500).
    Counts are exact integers and equal the oracle's on this scene (a decision within an ulp of the alpha / T thresholds
    could flip between v_exp_f32 and expf; none does here)."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from dogs_amd.diff_gaussian_rasterization import _C
    n, W, H = 2000, 160, 120
    s = small_scene(n, W, H, seed=17)
    c = s.camera.to(hip_device)
    bg = torch.tensor([0.1, 0.2, 0.3], device=hip_device)
    st = GaussianRasterizationSettings(image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, bg=bg,
                                       scale_modifier=1.0, depth_threshold=0.0, viewmatrix=c.world_to_camera,
                                       projmatrix=c.projective_matrix, sh_degree=3, campos=c.camera_center,
                                       prefiltered=False, debug=False, f_count=True)
    feats = torch.cat([s.dc, s.sh], dim=1).to(hip_device)
    old = _C.set_prefix_per_tile(prefix)
    try:
        count, score, img, radii = GaussianRasterizer(st)(means3D=s.means3D.to(hip_device), means2D=None,
                                                          opacities=s.opacities.to(hip_device), shs=feats,
                                                          scales=s.scales.to(hip_device),
                                                          rotations=s.rotations.to(hip_device))
    finally:
        _C.set_prefix_per_tile(old)
    col_o, radii_o, _, sto = oracle_forward(oracle, s, bg.cpu().numpy())
    cnt_o, score_o = sto.counts()
    np.testing.assert_array_equal(radii.cpu().numpy(), radii_o)
    assert np.abs(img.cpu().numpy() - col_o).max() < 5e-3
    cnt = count.cpu().numpy()
    assert count.dtype == torch.int32 and cnt.sum() > 0
    # every count equal: no (pixel, Gaussian) decision of this scene sits within an ulp of the 1/255 or T thresholds
    # where v_exp_f32 and expf could disagree (measured: 0 of 28,274 counted pixels differ; the inputs are fixed, so
    # the result is too)
    np.testing.assert_array_equal(cnt, cnt_o)
    np.testing.assert_allclose(score.cpu().numpy(), score_o, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("M", [1, 2, 3])
def test_row_prod_matches_torch_prod(hip_device, M):
    """dogs_amd.loss.row_prod (the scale regulariser's prod(dim=1) without prod_backward's host read) is bit-identical
    to torch.prod(x, 1) and its autograd gradient, on a wide value range, and with zeros (torch then takes its zero-safe
    form for every row)."""
    from dogs_amd.loss import row_prod
    g = torch.Generator().manual_seed(M)
    x = torch.exp(torch.randn((100_003, M), generator=g) * 4)
    x[5, 0] = 1e-30
    gout = torch.randn(x.shape[0], generator=g).to(hip_device)
    # zeros, then none again: the forward stamps its own call's value, so a stale stamp left in a reused word reads as
    # "no zero"
    for zeros in ((), ((77, M - 1),), ((1234, 0), (1234, M - 1), (9, 0)), ()):
        xx = x.clone()
        for r, c in zeros:
            xx[r, c] = 0.0
        a = xx.to(hip_device).requires_grad_(True)
        b = xx.to(hip_device).requires_grad_(True)
        pa, pb = torch.prod(a, dim=1), row_prod(b)
        assert torch.equal(pa, pb)
        (pa * gout).sum().backward()
        (pb * gout).sum().backward()
        assert torch.equal(a.grad, b.grad), zeros
        a.grad = b.grad = None
        torch.prod(a, dim=1).mean().backward()
        row_prod(b).mean().backward()
        assert torch.equal(a.grad, b.grad), zeros
