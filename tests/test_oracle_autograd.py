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


def dense_forward(s, lists, W, H, deg):
    """Returns (loss closure inputs): leaves dict and outputs (color, invdepth, ndc2, rgb, cov6)."""
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
    color = torch.zeros((3, H, W), dtype=f64)
    invd = torch.zeros((H, W), dtype=f64)
    tiles_x = (W + 15) // 16
    yy, xx = torch.meshgrid(torch.arange(16, dtype=f64), torch.arange(16, dtype=f64), indexing="ij")
    for t, gl in lists.items():
        x0, y0 = (t % tiles_x) * 16, (t // tiles_x) * 16
        pxs, pys = (xx + x0).reshape(-1), (yy + y0).reshape(-1)
        T = torch.ones(256, dtype=f64)
        live = torch.ones(256, dtype=torch.bool)
        C = torch.zeros((3, 256), dtype=f64)
        D = torch.zeros(256, dtype=f64)
        for g in gl:
            dx, dy = px[g] - pxs, py[g] - pys
            power = -0.5 * (ca[g] * dx * dx + cc[g] * dy * dy) - cb[g] * dx * dy
            alpha = torch.clamp_max(op[g] * torch.exp(power), 0.99)
            ok = live & (power.detach() <= 0) & (alpha.detach() >= 1.0 / 255.0)
            test_T = T * (1 - alpha)
            term = ok & (test_T.detach() < 1e-4)
            live = live & ~term
            ok = ok & ~term
            a = torch.where(ok, alpha, torch.zeros_like(alpha))
            C = C + rgb_c[g][:, None] * (a * T)[None, :]
            D = D + invz[g] * a * T
            T = torch.where(ok, test_T, T)
        inside = (pxs < W) & (pys < H)
        iy, ix = pys[inside].long(), pxs[inside].long()
        color = color.index_put((torch.arange(3)[:, None], iy[None, :], ix[None, :]), C[:, inside])
        invd = invd.index_put((iy, ix), D[inside])
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
