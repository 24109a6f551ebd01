"""Small boundary items of the `_C` table and the autograd wrapper:

* depth_threshold > 0 (diff_gaussian_rasterization/__init__.py:171-185): the backward's per-Gaussian depth output is
  the view-space z of every visible Gaussian (computeCov2DCUDA, backward.cu), and grad_means2D is the unscaled
  gradient times min(1, (z / thr)^2);
* `_C.fusedssim` / `_C.fusedssim_backward`, the conv.cu variant (conv.cu:1139-1194; exported by the reference
  extension, called nowhere in conerf): an [3,H,W] SSIM map with "same" zero padding and the 11x11 window as the 2-D
  constants G_ij = round(g_i g_j, 10) of the separable 1-D window g (conv.cu:8-140), and the exact gradient of
  sum(dL_dmap * map) w.r.t. img1 -- checked against a float64 torch restatement with those constants, differentiated
  by autograd (bar: 1e-5 absolute on the map, 1e-4 relative on the gradient: fp32 vs fp64 summation);
* `_C.count_gaussians` called directly (old rasterize_points.cu:148-233 signature) against the oracle.
"""
import numpy as np
import pytest
import torch

from raster_util import oracle_forward, rel_err, small_scene

pytestmark = pytest.mark.gpu


def _settings(c, W, H, bg, thr):
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    return GaussianRasterizationSettings(image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, bg=bg,
                                         scale_modifier=1.0, viewmatrix=c.world_to_camera,
                                         projmatrix=c.projective_matrix, sh_degree=3, campos=c.camera_center,
                                         prefiltered=False, debug=False, antialiasing=False, depth_threshold=thr)


def test_depth_threshold_scales_means2d_grad(hip_device):
    from diff_gaussian_rasterization import GaussianRasterizer
    from dogs_amd.diff_gaussian_rasterization import _C
    n, W, H = 3000, 192, 144
    s = small_scene(n, W, H, seed=41)
    c = s.camera.to(hip_device)
    bg = torch.zeros(3, device=hip_device)
    gc = torch.from_numpy(np.random.default_rng(2).standard_normal((3, H, W)).astype(np.float32)).to(hip_device)
    thr = 8.0   # the scene's depths span [2, 20]: some gradients scaled, some not
    grads = {}
    for t in (0.0, thr):
        leaf = {k: getattr(s, k).to(hip_device).clone().requires_grad_(True)
                for k in ("means3D", "opacities", "scales", "rotations", "dc", "sh")}
        m2d = torch.zeros_like(leaf["means3D"], requires_grad=True)
        img, radii, _ = GaussianRasterizer(_settings(c, W, H, bg, t))(
            leaf["means3D"], m2d, leaf["opacities"], dc=leaf["dc"], shs=leaf["sh"], scales=leaf["scales"],
            rotations=leaf["rotations"])
        (img * gc).sum().backward()
        grads[t] = (m2d.grad.clone(), leaf["means3D"].grad.clone(), radii)
    radii = grads[0.0][2]
    vis = radii > 0
    # view-space z of every Gaussian (viewmatrix = w2c^T, row-vector convention)
    m = s.means3D.to(hip_device)
    vm = c.world_to_camera
    z = m[:, 0] * vm[0, 2] + m[:, 1] * vm[1, 2] + m[:, 2] * vm[2, 2] + vm[3, 2]
    # the backward's depth output directly from the _C table
    e = torch.empty(0, device=hip_device)
    d = lambda t: t.to(hip_device).contiguous()  # noqa: E731
    out = _C.rasterize_gaussians(bg, d(s.means3D), e, d(s.opacities), d(s.scales), d(s.rotations), 1.0, e,
                                 c.world_to_camera, c.projective_matrix, c.tanfovx, c.tanfovy, H, W, d(s.dc), d(s.sh),
                                 3, c.camera_center, False, False, False)
    gr = _C.rasterize_gaussians_backward(bg, d(s.means3D), out[4], e, d(s.opacities), d(s.scales), d(s.rotations),
                                         1.0, e, c.world_to_camera, c.projective_matrix, c.tanfovx, c.tanfovy, gc,
                                         d(s.dc), d(s.sh), torch.zeros((1, H, W), device=hip_device), 3,
                                         c.camera_center, out[5], out[0], out[6], out[7], out[1], out[8], False, False)
    depth = gr[9].reshape(-1)
    torch.testing.assert_close(depth[vis], z[vis], rtol=1e-6, atol=1e-6)
    assert float(depth[~vis].abs().max()) == 0.0 if (~vis).any() else True
    scale = torch.minimum(torch.ones_like(depth), (depth / thr) ** 2)
    assert float((scale[vis] < 1).float().mean()) > 0.05 and float((scale[vis] == 1).float().mean()) > 0.05
    expect = grads[0.0][0] * scale.unsqueeze(-1)
    torch.testing.assert_close(grads[thr][0], expect, rtol=1e-6, atol=1e-12)
    # the other gradients are untouched by the threshold
    torch.testing.assert_close(grads[thr][1], grads[0.0][1], rtol=0, atol=0)


def _conv_ssim_restatement(img1, img2, C1, C2):
    """conv.cu fusedssimCUDA in float64: 2-D window constants round(g_i g_j, 10), zero padding (get_pix_value)."""
    x = np.arange(11) - 5
    g = np.exp(-(x ** 2) / (2 * 1.5 ** 2))
    g = (g / g.sum()).astype(np.float32).astype(np.float64)   # the G_0x float literals (ssim.cu:9-19)
    w2 = np.round(np.outer(g, g), 10)
    k = torch.from_numpy(w2).reshape(1, 1, 11, 11).expand(3, 1, 11, 11).contiguous()

    def conv(t):
        return torch.nn.functional.conv2d(t.unsqueeze(0), k, padding=5, groups=3)[0]
    mu1, mu2 = conv(img1), conv(img2)
    s11 = conv(img1 * img1) - mu1 * mu1
    s22 = conv(img2 * img2) - mu2 * mu2
    s12 = conv(img1 * img2) - mu1 * mu2
    Cn = 2 * mu1 * mu2 + C1
    Dn = 2 * s12 + C2
    An = mu1 * mu1 + mu2 * mu2 + C1
    Bn = s11 + s22 + C2
    return (Cn * Dn) / (An * Bn)


@pytest.mark.parametrize("H,W", [(37, 53), (96, 128)])
def test_conv_fusedssim_semantics(hip_device, H, W):
    from dogs_amd.diff_gaussian_rasterization import _C
    g = torch.Generator().manual_seed(H)
    img1 = torch.rand((3, H, W), generator=g)
    img2 = (img1 + 0.1 * torch.randn((3, H, W), generator=g)).clamp(0, 1)
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    m = _C.fusedssim(C1, C2, img1.to(hip_device), img2.to(hip_device))
    a = img1.double().requires_grad_(True)
    ref = _conv_ssim_restatement(a, img2.double(), C1, C2)
    assert m.shape == (3, H, W)
    np.testing.assert_allclose(m.cpu().numpy(), ref.detach().numpy(), rtol=0, atol=1e-5)
    dmap = torch.randn((3, H, W), generator=g)
    (ref * dmap.double()).sum().backward()
    d = _C.fusedssim_backward(C1, C2, img1.to(hip_device), img2.to(hip_device), dmap.to(hip_device))
    assert rel_err(d.cpu().numpy(), a.grad.numpy()) < 1e-4


def test_count_gaussians_direct_call(oracle, hip_device):
    from dogs_amd.diff_gaussian_rasterization import _C
    n, W, H = 1500, 128, 96
    s = small_scene(n, W, H, seed=23)
    c = s.camera.to(hip_device)
    bg = torch.tensor([0.3, 0.2, 0.1], device=hip_device)
    d = lambda t: t.to(hip_device).contiguous()  # noqa: E731
    e = torch.empty(0, device=hip_device)
    feats = torch.cat([s.dc, s.sh], dim=1)
    count, score, nr, color, radii, gb, bb, ib = _C.count_gaussians(
        bg, d(s.means3D), e, d(s.opacities), d(s.scales), d(s.rotations), 1.0, e, c.world_to_camera,
        c.projective_matrix, c.tanfovx, c.tanfovy, H, W, d(feats), 3, c.camera_center, False, False)
    col_o, radii_o, _, sto = oracle_forward(oracle, s, bg.cpu().numpy())
    cnt_o, score_o = sto.counts()
    assert isinstance(nr, int) and nr == sto.num_rendered
    np.testing.assert_array_equal(radii.cpu().numpy(), radii_o)
    assert np.abs(color.cpu().numpy() - col_o).max() < 5e-3
    cnt = count.cpu().numpy()
    assert count.dtype == torch.int32 and cnt.sum() > 0
    np.testing.assert_array_equal(cnt, cnt_o)   # as test_gpu_aux.py::test_count_mode_matches_oracle
    np.testing.assert_allclose(score.cpu().numpy(), score_o, rtol=1e-4, atol=1e-6)
    assert gb.numel() == 0 and bb.numel() == 0 and ib.numel() == 0
