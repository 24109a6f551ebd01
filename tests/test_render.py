"""render() (conerf/render/gaussian_render.py:18-158) through dogs_amd.render: the result dict and its routing of
model attributes into the rasterizer (separate_sh, full features, override colours, Python-side SH and covariance,
trained exposure, clamp), against direct calls of this package's GaussianRasterizer and, for the Python-side SH,
the reference's sh_utils.eval_sh values (fp32 tolerance 1e-5 written in the test).  The CPU tests check eval_sh
against a direct restatement of sh_utils.py:57-112 and that render refuses CPU tensors (no fallback)."""
import math
import types

import pytest
import torch

from dogs_amd.render import eval_sh, render


def _eval_sh_ref(deg, sh, d):   # sh_utils.py:57-112 written out term by term
    C0, C1 = 0.28209479177387814, 0.4886025119029199
    C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
    C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
          1.445305721320277, -0.5900435899266435]
    r = C0 * sh[..., 0]
    if deg > 0:
        x, y, z = d[..., 0:1], d[..., 1:2], d[..., 2:3]
        r = r - C1 * y * sh[..., 1] + C1 * z * sh[..., 2] - C1 * x * sh[..., 3]
        if deg > 1:
            xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
            r = (r + C2[0] * xy * sh[..., 4] + C2[1] * yz * sh[..., 5] + C2[2] * (2.0 * zz - xx - yy) * sh[..., 6]
                 + C2[3] * xz * sh[..., 7] + C2[4] * (xx - yy) * sh[..., 8])
            if deg > 2:
                r = (r + C3[0] * y * (3 * xx - yy) * sh[..., 9] + C3[1] * xy * z * sh[..., 10]
                     + C3[2] * y * (4 * zz - xx - yy) * sh[..., 11] + C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[..., 12]
                     + C3[4] * x * (4 * zz - xx - yy) * sh[..., 13] + C3[5] * z * (xx - yy) * sh[..., 14]
                     + C3[6] * x * (xx - 3 * yy) * sh[..., 15])
    return r


def test_eval_sh_matches_the_reference_expression():
    g = torch.Generator().manual_seed(0)
    sh = torch.randn(100, 3, 16, generator=g)
    d = torch.nn.functional.normalize(torch.randn(100, 3, generator=g), dim=1)
    for deg in range(4):
        assert torch.equal(eval_sh(deg, sh, d), _eval_sh_ref(deg, sh, d))
    with pytest.raises(ValueError):
        eval_sh(4, torch.zeros(1, 3, 25), d[:1])


def _build_cov(scales, rot, mod=1.0):   # GaussianSplatModel.get_covariance: strip_symmetric(R S S^T R^T)
    r, x, y, z = rot.unbind(-1)
    R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
                     2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
                     2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1).view(-1, 3, 3)
    L = R @ torch.diag_embed(mod * scales)
    S = L @ L.transpose(1, 2)
    return torch.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1], S[:, 1, 2], S[:, 2, 2]], -1)


def _model(s, dev, deg=3):
    m = types.SimpleNamespace()
    m.get_xyz = s.means3D.to(dev).requires_grad_(True)
    m.get_opacity = s.opacities.to(dev)
    m.get_scaling = s.scales.to(dev)
    m.get_quaternion = s.rotations.to(dev)
    m.get_features_dc = s.dc.to(dev)
    m.get_features_rest = s.sh.to(dev)
    m.get_features = torch.cat([m.get_features_dc, m.get_features_rest], dim=1)
    m.active_sh_degree = deg
    m.max_sh_degree = 3
    m.get_covariance = lambda mod=1.0: _build_cov(m.get_scaling, m.get_quaternion, mod)
    expo = torch.eye(3, 4, device=dev)
    expo[:3, :3] *= 0.9
    expo[:, 3] = torch.tensor([0.01, -0.02, 0.03], device=dev)
    m.get_exposure_from_id = lambda i: expo
    return m


def _cam(s, dev):
    c = s.camera.to(dev)
    c.image_index = 0
    return c


def _direct(s, dev, bg, **kw):
    from dogs_amd.diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    c = s.camera.to(dev)
    rs = GaussianRasterizationSettings(c.height, c.width, math.tan(c.fov_x * 0.5), math.tan(c.fov_y * 0.5), bg, 1.0,
                                       c.world_to_camera, c.projective_matrix, 3, c.camera_center, False, False,
                                       False, 0.0)
    m2d = torch.zeros_like(s.means3D.to(dev), requires_grad=True)
    img, radii, depth = GaussianRasterizer(rs)(means3D=s.means3D.to(dev), means2D=m2d, opacities=s.opacities.to(dev),
                                               **kw)
    return img.clamp(0, 1), radii, depth


def test_render_refuses_cpu_tensors():
    from raster_util import small_scene
    s = small_scene(50, 32, 32, seed=1)
    cfg = types.SimpleNamespace(debug=False, compute_cov3D_python=False, convert_SHs_python=False)
    with pytest.raises((RuntimeError, ImportError, AssertionError)):
        render(_model(s, "cpu"), _cam(s, "cpu"), cfg, torch.zeros(3), device="cpu")


@pytest.mark.gpu
def test_render_routes_like_the_reference(hip_device):
    from raster_util import small_scene
    dev = hip_device
    s = small_scene(3000, 160, 120, seed=5)
    bg = torch.tensor([0.1, 0.2, 0.3], device=dev)
    cfg = types.SimpleNamespace(debug=False, compute_cov3D_python=False, convert_SHs_python=False)
    ref_img, ref_radii, ref_depth = _direct(s, dev, bg, dc=s.dc.to(dev), shs=s.sh.to(dev),
                                            scales=s.scales.to(dev), rotations=s.rotations.to(dev))
    for sep in (True, False):
        m = _model(s, dev)
        out = render(m, _cam(s, dev), cfg, bg, separate_sh=sep, device=dev)
        assert torch.equal(out["rendered_image"], ref_img)
        assert torch.equal(out["radii"], ref_radii) and torch.equal(out["depth"], ref_depth)
        assert torch.equal(out["visibility_filter"], ref_radii > 0)
        assert out["scaling"] is m.get_scaling
        (out["rendered_image"].sum()).backward()
        assert out["screen_space_points"].grad is not None and out["screen_space_points"].grad.abs().sum() > 0
        assert m.get_xyz.grad is not None
    # override colours
    colors = torch.rand(3000, 3, device=dev)
    img, _, _ = _direct(s, dev, bg, colors_precomp=colors, scales=s.scales.to(dev), rotations=s.rotations.to(dev))
    out = render(_model(s, dev), _cam(s, dev), cfg, bg, override_color=colors, device=dev)
    assert torch.equal(out["rendered_image"], img)
    # Python-side covariance
    cfg_cov = types.SimpleNamespace(debug=False, compute_cov3D_python=True, convert_SHs_python=False)
    m = _model(s, dev)
    img, _, _ = _direct(s, dev, bg, dc=s.dc.to(dev), shs=s.sh.to(dev), cov3D_precomp=m.get_covariance(1.0))
    out = render(m, _cam(s, dev), cfg_cov, bg, separate_sh=True, device=dev)
    assert torch.equal(out["rendered_image"], img) and out["scaling"] is None
    # Python-side SH: the same colours the rasterizer evaluates, within fp32 rounding (1e-5)
    cfg_sh = types.SimpleNamespace(debug=False, compute_cov3D_python=False, convert_SHs_python=True)
    out = render(_model(s, dev), _cam(s, dev), cfg_sh, bg, device=dev)
    assert (out["rendered_image"] - ref_img).abs().max().item() < 1e-5
    # trained exposure on the unclamped rasterizer output, then the clamp
    m = _model(s, dev)
    out = render(m, _cam(s, dev), cfg, bg, separate_sh=True, use_trained_exposure=True, device=dev)
    from dogs_amd.diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    c = s.camera.to(dev)
    rs = GaussianRasterizationSettings(c.height, c.width, math.tan(c.fov_x * 0.5), math.tan(c.fov_y * 0.5), bg, 1.0,
                                       c.world_to_camera, c.projective_matrix, 3, c.camera_center, False, False,
                                       False, 0.0)
    img0, _, _ = GaussianRasterizer(rs)(means3D=s.means3D.to(dev), means2D=torch.zeros_like(s.means3D.to(dev)),
                                        opacities=s.opacities.to(dev), dc=s.dc.to(dev), shs=s.sh.to(dev),
                                        scales=s.scales.to(dev), rotations=s.rotations.to(dev))
    e = m.get_exposure_from_id(0)
    want = (torch.matmul(img0.permute(1, 2, 0), e[:3, :3]).permute(2, 0, 1) + e[:3, 3, None, None]).clamp(0, 1)
    assert torch.equal(out["rendered_image"], want)
