"""Independent check of the oracle BACKWARD: a dense float64 PyTorch restatement of the rasterizer forward
(projection, EWA covariance, SH colour, front-to-back compositing over the oracle's per-tile lists), differentiated
with torch autograd, must give the gradients the oracle's restatement of the reference bucket backward
(backward.cu:23-658) produces.  Background 0: with bg != 0 the reference backward double-counts the background
term (a replicated quirk, DESIGN.md "Parity"), which autograd of the true forward does not.

Reference conventions restated here: auxiliary.h:40-172 (ndc2Pix, transforms, in_frustum), forward.cu:24-76 (SH),
:114-243 (cov2D / cov3D), :441-591 (compositing rules).  CPU only.
"""
import numpy as np
import pytest
import torch

from raster_util import oracle_forward, small_scene

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
SH_C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
         1.445305721320277, -0.5900435899266435]


def sh_rgb(deg, dc, sh, dirs):
    x, y, z = dirs[:, 0:1], dirs[:, 1:2], dirs[:, 2:3]
    r = SH_C0 * dc[:, 0]
    if deg > 0:
        r = r - SH_C1 * y * sh[:, 0] + SH_C1 * z * sh[:, 1] - SH_C1 * x * sh[:, 2]
    if deg > 1:
        xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
        r = (r + SH_C2[0] * xy * sh[:, 3] + SH_C2[1] * yz * sh[:, 4] + SH_C2[2] * (2 * zz - xx - yy) * sh[:, 5]
             + SH_C2[3] * xz * sh[:, 6] + SH_C2[4] * (xx - yy) * sh[:, 7])
    if deg > 2:
        r = (r + SH_C3[0] * y * (3 * xx - yy) * sh[:, 8] + SH_C3[1] * xy * z * sh[:, 9]
             + SH_C3[2] * y * (4 * zz - xx - yy) * sh[:, 10] + SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 11]
             + SH_C3[4] * x * (4 * zz - xx - yy) * sh[:, 12] + SH_C3[5] * z * (xx - yy) * sh[:, 13]
             + SH_C3[6] * x * (xx - 3 * yy) * sh[:, 14])
    return r + 0.5


def dense_forward(s, lists, W, H, deg, bg=None, extra=None, antialiasing=False):
    """Returns (loss closure inputs): leaves dict and outputs (color, invdepth, ndc2, rgb, cov6).  bg: the colour
    behind the splats (final colour + T_final bg, forward.cu:575-580); extra (a dict) receives the per-pixel final
    transmittance `T_final` [H,W], `qlog` = sum over the pixel's accepted splats of -log(1 - alpha) [H,W] and the
    number of pixels that reached the T < 1e-4 stop, `stopped_pixels`."""
    f64 = torch.float64
    c = s.camera
    V = c.world_to_camera.to(f64)          # rows: p_view = [p,1] @ V  (transformPoint4x3)
    Pm = c.projective_matrix.to(f64)
    leaves = {k: getattr(s, k).to(f64).clone().requires_grad_(True)
              for k in ("means3D", "scales", "rotations", "opacities", "dc", "sh")}
    m = leaves["means3D"]
    ones = torch.ones((m.shape[0], 1), dtype=f64)
    ph = torch.cat([m, ones], 1)
    pv = (ph @ V)[:, :3]
    pp = ph @ Pm
    ndc = pp[:, :3] / (pp[:, 3:4] + 1e-7)
    ndc2 = ndc[:, :2]
    ndc2.retain_grad()
    px = ((ndc2[:, 0] + 1.0) * W - 1.0) * 0.5
    py = ((ndc2[:, 1] + 1.0) * H - 1.0) * 0.5
    # cov3D = R S S R^T from the (already normalised) quaternion, no in-kernel normalisation (forward.cu:128)
    q = leaves["rotations"]
    r_, x_, y_, z_ = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.stack([1 - 2 * (y_ * y_ + z_ * z_), 2 * (x_ * y_ - r_ * z_), 2 * (x_ * z_ + r_ * y_),
                     2 * (x_ * y_ + r_ * z_), 1 - 2 * (x_ * x_ + z_ * z_), 2 * (y_ * z_ - r_ * x_),
                     2 * (x_ * z_ - r_ * y_), 2 * (y_ * z_ + r_ * x_), 1 - 2 * (x_ * x_ + y_ * y_)], 1).reshape(-1, 3, 3)
    L = R * leaves["scales"][:, None, :]
    Sig = L @ L.transpose(1, 2)
    cov6 = torch.stack([Sig[:, 0, 0], Sig[:, 0, 1], Sig[:, 0, 2], Sig[:, 1, 1], Sig[:, 1, 2], Sig[:, 2, 2]], 1)
    cov6.retain_grad()
    S6 = cov6
    Sg = torch.stack([S6[:, 0], S6[:, 1], S6[:, 2], S6[:, 1], S6[:, 3], S6[:, 4], S6[:, 2], S6[:, 4], S6[:, 5]],
                     1).reshape(-1, 3, 3)
    # EWA (forward.cu:114-165): clamp of x/z, y/z to 1.3 tan(fov); J; W = rotation part
    fx = W / (2.0 * c.tanfovx)
    fy = H / (2.0 * c.tanfovy)
    limx, limy = 1.3 * c.tanfovx, 1.3 * c.tanfovy
    tz = pv[:, 2]
    tx = torch.clamp(pv[:, 0] / tz, -limx, limx) * tz
    ty = torch.clamp(pv[:, 1] / tz, -limy, limy) * tz
    zero = torch.zeros_like(tz)
    J = torch.stack([fx / tz, zero, -fx * tx / (tz * tz), zero, fy / tz, -fy * ty / (tz * tz)], 1).reshape(-1, 2, 3)
    Rwc = V[:3, :3].T
    cam = Rwc @ Sg @ Rwc.T
    c2 = J @ cam @ J.transpose(1, 2)
    cxx, cxy, cyy = c2[:, 0, 0] + 0.3, c2[:, 0, 1], c2[:, 1, 1] + 0.3
    det = cxx * cyy - cxy * cxy
    ca, cb, cc = cyy / det, -cxy / det, cxx / det
    cen = c.camera_center.to(f64)
    dirs = m - cen[None, :]
    dirs = dirs / dirs.norm(dim=1, keepdim=True)
    rgb = sh_rgb(deg, leaves["dc"], leaves["sh"], dirs)
    rgb_c = torch.clamp_min(rgb, 0.0)
    rgb_c.retain_grad()
    invz = 1.0 / pv[:, 2]
    op = leaves["opacities"][:, 0]
    if antialiasing:
        # the opacity compensation of the 0.3 px dilation (forward.cu:218-233): sqrt(max(2.5e-5, det / det+)).  Its
        # gradient is the reference's, not the exact one: backward.cu:212-246 evaluates d(det / det+)/d(xx, xy, yy) --
        # derived for the undilated entries -- at the DILATED ones (it adds h_var first).  So the value is the true
        # scaling and the gradient flows through r(xx + 0.3, xy, yy + 0.3), the same function at the shifted point
        # (the reference's second quirk; exact autograd of the true forward puts dcov3D 64% off it), and none when
        # the clamp holds.
        def ratio(a_, b_, c_):
            return (a_ * c_ - b_ * b_) / ((a_ + 0.3) * (c_ + 0.3) - b_ * b_)
        r0 = ratio(c2[:, 0, 0], c2[:, 0, 1], c2[:, 1, 1])
        hs = torch.sqrt(torch.clamp_min(r0, 0.000025)).detach()
        rs = ratio(c2[:, 0, 0] + 0.3, c2[:, 0, 1], c2[:, 1, 1] + 0.3)
        live = (r0.detach() > 0.000025).to(rs.dtype)
        op = op * (hs + live * (rs - rs.detach()) / (2.0 * hs))
    color = torch.zeros((3, H, W), dtype=f64)
    invd = torch.zeros((H, W), dtype=f64)
    tfin = torch.ones((H, W), dtype=f64)
    qlog = torch.zeros((H, W), dtype=f64)
    nstop = 0
    counts = torch.zeros(m.shape[0], dtype=torch.int64)
    bgv = None if bg is None else torch.as_tensor(bg, dtype=f64)
    tiles_x = (W + 15) // 16
    yy, xx = torch.meshgrid(torch.arange(16, dtype=f64), torch.arange(16, dtype=f64), indexing="ij")
    for t, gl in lists.items():
        x0, y0 = (t % tiles_x) * 16, (t // tiles_x) * 16
        pxs, pys = (xx + x0).reshape(-1), (yy + y0).reshape(-1)
        T = torch.ones(256, dtype=f64)
        live = torch.ones(256, dtype=torch.bool)
        C = torch.zeros((3, 256), dtype=f64)
        D = torch.zeros(256, dtype=f64)
        Q = torch.zeros(256, dtype=f64)
        stop = torch.zeros(256, dtype=torch.bool)
        in_img = (pxs < W) & (pys < H)
        for g in gl:
            dx, dy = px[g] - pxs, py[g] - pys
            power = -0.5 * (ca[g] * dx * dx + cc[g] * dy * dy) - cb[g] * dx * dy
            alpha = torch.clamp_max(op[g] * torch.exp(power), 0.99)
            ok = live & (power.detach() <= 0) & (alpha.detach() >= 1.0 / 255.0)
            test_T = T * (1 - alpha)
            term = ok & (test_T.detach() < 1e-4)
            stop = stop | term
            live = live & ~term
            ok = ok & ~term
            counts[g] += int((ok & in_img).sum())
            a = torch.where(ok, alpha, torch.zeros_like(alpha))
            C = C + rgb_c[g][:, None] * (a * T)[None, :]
            D = D + invz[g] * a * T
            Q = Q - torch.log1p(-a)
            T = torch.where(ok, test_T, T)
        if bgv is not None:
            C = C + bgv[:, None] * T[None, :]
        inside = (pxs < W) & (pys < H)
        iy, ix = pys[inside].long(), pxs[inside].long()
        color = color.index_put((torch.arange(3)[:, None], iy[None, :], ix[None, :]), C[:, inside])
        invd = invd.index_put((iy, ix), D[inside])
        tfin = tfin.index_put((iy, ix), T[inside])
        nstop += int(stop[inside].sum())
        qlog = qlog.index_put((iy, ix), Q[inside])
    if extra is not None:
        extra["T_final"], extra["qlog"], extra["stopped_pixels"] = tfin, qlog, nstop
        extra["counts"] = counts.numpy()  # accepted pixels per Gaussian: LightGaussian's count (old forward.cu:485)
    return leaves, color, invd, ndc2, rgb_c, cov6


@pytest.mark.parametrize("n,W,H,deg,seed", [(6, 40, 36, 3, 1), (24, 48, 40, 2, 2), (40, 64, 48, 3, 4)])
def test_oracle_backward_matches_autograd(oracle, n, W, H, deg, seed):
    s = small_scene(n, W, H, seed=seed)
    s.opacities = torch.clamp(s.opacities, max=0.9)      # keep alpha away from the 0.99 clamp
    col_o, radii_o, inv_o, st = oracle_forward(oracle, s, (0, 0, 0), deg=deg)
    tiles, gids, _ = st.sorted_list()
    lists = {}
    for t, g in zip(tiles.tolist(), gids.tolist()):
        lists.setdefault(t, []).append(g)
    leaves, color, invd, ndc2, rgb_c, cov6 = dense_forward(s, lists, W, H, deg)
    np.testing.assert_allclose(color.detach().numpy(), col_o, atol=2e-5)
    rng = np.random.default_rng(seed)
    gcol = rng.standard_normal((3, H, W))
    ginv = 0.1 * rng.standard_normal((H, W))
    loss = (color * torch.from_numpy(gcol)).sum() + (invd * torch.from_numpy(ginv)).sum()
    loss.backward()
    go = st.backward(gcol.astype(np.float32), ginv.astype(np.float32))
    vis = radii_o > 0
    checks = {
        "dmeans3D": leaves["means3D"].grad, "dscales": leaves["scales"].grad, "drot": leaves["rotations"].grad,
        "dopacity": leaves["opacities"].grad, "ddc": leaves["dc"].grad, "dsh": leaves["sh"].grad,
        "dcolors": rgb_c.grad, "dcov3D": cov6.grad,
    }
    for name, ref in checks.items():
        got = go[name][vis]
        ref = ref.detach().numpy()[vis].reshape(got.shape)
        err = np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-12)
        assert err < 2e-4, f"{name}: rel err {err}"
    ref2 = ndc2.grad.detach().numpy()[vis]
    got2 = go["dmeans2D"][vis, :2]
    err = np.linalg.norm(got2 - ref2) / np.linalg.norm(ref2)
    assert err < 2e-4, f"dmeans2D: rel err {err}"


def reference_radii(s, W, H):
    """forward.cu:196-266 restated in float64: in_frustum (view z > 0.2, auxiliary.h:151-172), the dilated EWA
    covariance, det != 0, my_radius = ceil(3 sqrt(max(lambda1, lambda2))) with the eigenvalue floor of 0.1, the
    projected centre ndc2Pix, and radius 0 when getRect's rectangle is empty (auxiliary.h:45-55; its int() truncation
    equals floor after the clamp at 0).  Returns (radii int64 [P], means2D float64 [P, 2])."""
    f64 = torch.float64
    c = s.camera
    V = c.world_to_camera.to(f64)
    Pm = c.projective_matrix.to(f64)
    m = s.means3D.to(f64)
    ph = torch.cat([m, torch.ones((m.shape[0], 1), dtype=f64)], 1)
    pv = (ph @ V)[:, :3]
    pp = ph @ Pm
    ndc = pp[:, :3] / (pp[:, 3:4] + 1e-7)
    px = ((ndc[:, 0] + 1.0) * W - 1.0) * 0.5
    py = ((ndc[:, 1] + 1.0) * H - 1.0) * 0.5
    q = s.rotations.to(f64)
    r_, x_, y_, z_ = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.stack([1 - 2 * (y_ * y_ + z_ * z_), 2 * (x_ * y_ - r_ * z_), 2 * (x_ * z_ + r_ * y_),
                     2 * (x_ * y_ + r_ * z_), 1 - 2 * (x_ * x_ + z_ * z_), 2 * (y_ * z_ - r_ * x_),
                     2 * (x_ * z_ - r_ * y_), 2 * (y_ * z_ + r_ * x_), 1 - 2 * (x_ * x_ + y_ * y_)], 1).reshape(-1, 3, 3)
    L = R * s.scales.to(f64)[:, None, :]
    Sg = L @ L.transpose(1, 2)
    fx, fy = W / (2.0 * c.tanfovx), H / (2.0 * c.tanfovy)
    limx, limy = 1.3 * c.tanfovx, 1.3 * c.tanfovy
    tz = pv[:, 2]
    tx = torch.clamp(pv[:, 0] / tz, -limx, limx) * tz
    ty = torch.clamp(pv[:, 1] / tz, -limy, limy) * tz
    zero = torch.zeros_like(tz)
    J = torch.stack([fx / tz, zero, -fx * tx / (tz * tz), zero, fy / tz, -fy * ty / (tz * tz)], 1).reshape(-1, 2, 3)
    Rwc = V[:3, :3].T
    c2 = J @ (Rwc @ Sg @ Rwc.T) @ J.transpose(1, 2)
    a, b, cc = c2[:, 0, 0] + 0.3, c2[:, 0, 1], c2[:, 1, 1] + 0.3
    det = a * cc - b * b
    mid = 0.5 * (a + cc)
    l1 = mid + torch.sqrt(torch.clamp_min(mid * mid - det, 0.1))
    l2 = mid - torch.sqrt(torch.clamp_min(mid * mid - det, 0.1))
    rad = torch.ceil(3.0 * torch.sqrt(torch.maximum(l1, l2)))
    gx, gy = (W + 15) // 16, (H + 15) // 16
    x0 = torch.clamp((px - rad) / 16, min=0).floor().clamp(max=gx)
    x1 = torch.clamp((px + rad + 15) / 16, min=0).floor().clamp(max=gx)
    y0 = torch.clamp((py - rad) / 16, min=0).floor().clamp(max=gy)
    y1 = torch.clamp((py + rad + 15) / 16, min=0).floor().clamp(max=gy)
    ok = (pv[:, 2] > 0.2) & (det != 0) & ((x1 - x0) * (y1 - y0) > 0)
    radii = torch.where(ok, rad, torch.zeros_like(rad)).numpy().astype(np.int64)
    return radii, torch.stack([px, py], 1).numpy()


@pytest.mark.parametrize("n,W,H,seed,k", [(60, 64, 48, 5, 1.0), (1200, 64, 48, 8, 7.0), (3000, 256, 192, 3, 1.0),
                                         (20000, 800, 600, 4, 1.0)])
def test_reference_radii_equal_oracle(oracle, n, W, H, seed, k):
    """The float64 restatement of the reference's culling and radius rules gives the oracle's radii exactly (0 of
    24,570 Gaussians differed when this was written)."""
    s = small_scene(n, W, H, seed=seed)
    s.scales = (s.scales * k).contiguous()
    _, radii_o, _, _ = oracle_forward(oracle, s, (0, 0, 0), deg=3)
    r64, _ = reference_radii(s, W, H)
    np.testing.assert_array_equal(r64, radii_o.astype(np.int64))


def rect_tile_lists(s, radii, means2D, W, H):
    """The reference's tile lists without its precise per-tile cull and without its key sort: every rendered Gaussian
    (radii > 0) in every tile of its getRect rectangle (auxiliary.h getRect: the 3-sigma radius around the projected
    centre, in 16 x 16 tiles), ordered by view depth computed here in float64 (ties: Gaussian index).  The cull only
    drops tiles no pixel of which accepts the splat (alpha < 1/255 everywhere), so compositing over these lists must
    give the reference's image and gradients: an anchor that shares no keying, culling or sorting code with the
    oracle: the radii and centres come from reference_radii (float64), checked equal to the oracle's first."""
    tx, ty = (W + 15) // 16, (H + 15) // 16
    c = s.camera
    ph = torch.cat([s.means3D.double(), torch.ones((s.means3D.shape[0], 1), dtype=torch.float64)], 1)
    z = (ph @ c.world_to_camera.double())[:, 2].numpy()
    lists = {}
    for g in np.lexsort((np.arange(len(z)), z)):
        r = int(radii[g])
        if r <= 0:
            continue
        px, py = float(means2D[g, 0]), float(means2D[g, 1])
        x0 = min(tx, max(0, int(np.floor((px - r) / 16)))); x1 = min(tx, max(0, int(np.floor((px + r + 15) / 16))))
        y0 = min(ty, max(0, int(np.floor((py - r) / 16)))); y1 = min(ty, max(0, int(np.floor((py + r + 15) / 16))))
        for yy in range(y0, y1):
            for xx in range(x0, x1):
                lists.setdefault(yy * tx + xx, []).append(int(g))
    return lists


@pytest.mark.parametrize("n,W,H,deg,seed,bg,aa", [(60, 64, 48, 3, 5, (0.3, 0.6, 0.9), False),
                                                 (120, 80, 64, 3, 6, (1.0, 0.5, 0.0), False),
                                                 (40, 64, 48, 2, 7, (0.0, 0.0, 0.0), False),
                                                 (150, 64, 48, 3, 9, (0.5, 0.5, 0.5), True),   # anti-aliasing
                                                 (1200, 64, 48, 3, 8, (0.2, 0.4, 0.6), False)])  # pixels saturate
def test_oracle_backward_matches_autograd_uncull_bg(oracle, n, W, H, deg, seed, bg, aa):
    """The stronger anchor (bg = 0 only, the oracle's own lists): the dense float64 forward over the
    uncull rect lists above, with a background, differentiated by autograd, against the oracle's restatement of the
    reference backward.  The reference counts the background twice in dL/dalpha (its accumulated colour starts from
    the final colour including T_final bg, and dL/dalpha also gets -T_final (bg . g) / (1 - alpha); DESIGN.md
    "Parity"), so the autograd loss carries that second count explicitly: sum over pixels of
    -T_final (bg . g) * sum over the pixel's accepted splats of -log(1 - alpha), T_final and g held constant, whose
    alpha-derivative is exactly the extra term.  Images within 2e-5, every gradient within 2e-4 relative."""
    s = small_scene(n, W, H, seed=seed)
    s.opacities = torch.clamp(s.opacities, max=0.9)
    if n >= 1200:  # dense, large and nearly opaque: ~570 of the 3072 pixels reach the T < 1e-4 stop
        s.opacities = torch.full_like(s.opacities, 0.95)
        s.scales = (s.scales * 7.0).contiguous()
    col_o, radii_o, inv_o, st = oracle_forward(oracle, s, bg, deg=deg, antialiasing=aa)
    r64, m64 = reference_radii(s, W, H)
    np.testing.assert_array_equal(r64, radii_o.astype(np.int64))
    lists = rect_tile_lists(s, r64, m64, W, H)
    extra = {}
    leaves, color, invd, ndc2, rgb_c, cov6 = dense_forward(s, lists, W, H, deg, bg=bg, extra=extra, antialiasing=aa)
    np.testing.assert_allclose(color.detach().numpy(), col_o, atol=2e-5)
    np.testing.assert_allclose(invd.detach().numpy(), inv_o[0], atol=2e-5)
    if n >= 1200:  # the dense case reaches the T < 1e-4 stop (forward.cu:560-566) in many pixels
        assert extra["stopped_pixels"] > 100
    # the precise per-tile cull is conservative, checked directly: every (tile, Gaussian) pair of the rect lists that
    # the oracle's keying dropped has no pixel of that tile where the splat reaches alpha >= 1/255 with power <= 0
    t_o, i_o, _ = st.sorted_list()
    kept = set(zip(t_o.tolist(), i_o.tolist()))
    g64 = st.geom()
    co, xy = g64["conic_opacity"].astype(np.float64), g64["means2D"].astype(np.float64)
    gx = (W + 15) // 16
    yy, xx = np.meshgrid(np.arange(16.0), np.arange(16.0), indexing="ij")
    dropped = 0
    for t, gl in lists.items():
        x0, y0 = (t % gx) * 16, (t // gx) * 16
        for g in gl:
            if (t, g) in kept:
                continue
            dropped += 1
            dx, dy = xy[g, 0] - (xx + x0), xy[g, 1] - (yy + y0)
            power = -0.5 * (co[g, 0] * dx * dx + co[g, 2] * dy * dy) - co[g, 1] * dx * dy
            alpha = np.minimum(0.99, co[g, 3] * np.exp(power))
            assert not np.any((power <= 0) & (alpha >= (1.0 / 255.0) * (1 + 1e-5))), (t, g)
    assert dropped > 0 or n < 100
    # the count mode's per-Gaussian accepted-pixel counts (old forward.cu:455-490) over the same independent lists
    cnt_o, _ = st.counts()
    cnt64 = extra["counts"]
    assert np.abs(cnt_o.astype(np.int64) - cnt64).max() <= 1 and (cnt_o == cnt64).mean() > 0.98
    rng = np.random.default_rng(seed)
    gcol = rng.standard_normal((3, H, W))
    ginv = 0.1 * rng.standard_normal((H, W))
    g_t = torch.from_numpy(gcol)
    bg_dot = (torch.as_tensor(bg, dtype=torch.float64)[:, None, None] * g_t).sum(0)
    quirk = (-(extra["T_final"].detach() * bg_dot) * extra["qlog"]).sum()
    loss = (color * g_t).sum() + (invd * torch.from_numpy(ginv)).sum() + quirk
    loss.backward()
    go = st.backward(gcol.astype(np.float32), ginv.astype(np.float32))
    vis = radii_o > 0
    checks = {
        "dmeans3D": leaves["means3D"].grad, "dscales": leaves["scales"].grad, "drot": leaves["rotations"].grad,
        "dopacity": leaves["opacities"].grad, "ddc": leaves["dc"].grad, "dsh": leaves["sh"].grad,
        "dcolors": rgb_c.grad, "dcov3D": cov6.grad,
    }
    for name, ref in checks.items():
        got = go[name][vis]
        ref = ref.detach().numpy()[vis].reshape(got.shape)
        err = np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-12)
        assert err < 2e-4, f"{name}: rel err {err}"
    ref2 = ndc2.grad.detach().numpy()[vis]
    got2 = go["dmeans2D"][vis, :2]
    assert np.linalg.norm(got2 - ref2) / np.linalg.norm(ref2) < 2e-4
