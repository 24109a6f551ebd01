"""Pin the CPU oracle (oracle/gs_oracle.c, oracle/aux_oracle.c) against the golden vectors of tests/golden/.

golden_sh_cov / golden_ssim hold outputs of the REFERENCE's own Python (tests/golden/make_golden.py):
  * preprocess RGB == clamp_min(eval_sh(deg, ...) + 0.5, 0)   (gaussian_render.py:87-102, sh_utils.py:57)
  * preprocess cov3D == L L^T, L = rotation_mat_left_multiply_scale_mat (utils.py:70, model :111-117)
  * fused-ssim "same" value / dL/dimg1 == ssim_torch.ssim and its autograd (ssim_torch.py:82)
golden_raster_* are frozen oracle outputs (regression: keys/radii/counts bit-exact, floats to 1e-6).
CPU only: no GPU and no reference import at test time.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return dict(np.load(os.path.join(G, name), allow_pickle=False))


def _forward(a, deg, bg=(0.0, 0.0, 0.0), aa=False):
    return O.forward(a["means3D"], a["opacities"], a["viewmatrix"], a["projmatrix"], a["campos"], float(a["tanfovx"]),
                     float(a["tanfovy"]), int(a["H"]), int(a["W"]), np.asarray(bg, np.float32), dc=a["dc"], sh=a["sh"],
                     scales=a["scales"], rotations=a["rotations"], sh_degree=deg, antialiasing=aa)


@pytest.mark.parametrize("deg", [0, 1, 2, 3])
def test_sh_colour_matches_reference_eval_sh(oracle, deg):
    a = _load("golden_sh_cov.npz")
    _, radii, _, st = _forward(a, deg)
    vis = radii > 0
    assert vis.sum() > 100
    rgb = st.geom()["rgb"]
    np.testing.assert_allclose(rgb[vis], a[f"rgb_deg{deg}"][vis], rtol=0, atol=2e-6)


def test_cov3d_matches_reference_LLt(oracle):
    a = _load("golden_sh_cov.npz")
    _, radii, _, st = _forward(a, 3)
    vis = radii > 0
    cov = st.geom()["cov3D"]
    ref = a["cov3D"]
    scale = np.abs(ref[vis]).max(axis=1, keepdims=True)
    np.testing.assert_allclose(cov[vis] / scale, ref[vis] / scale, rtol=0, atol=2e-6)


@pytest.mark.parametrize("tag", ["a", "b"])
def test_ssim_matches_reference_ssim_torch(oracle, tag):
    a = _load("golden_ssim.npz")
    img1, img2 = a[f"{tag}_img1"], a[f"{tag}_img2"]
    mp, d1, d2, d3 = O.ssim_forward(img1, img2)
    assert abs(float(mp.mean(dtype=np.float64)) - float(a[f"{tag}_value"])) < 2e-6
    dmap = np.full_like(mp, 1.0 / mp.size)
    g = O.ssim_backward(img1, img2, dmap, d1, d2, d3)
    ref = a[f"{tag}_grad"]
    assert np.abs(g - ref).max() <= 1e-4 * np.abs(ref).max()


@pytest.mark.parametrize("tag", ["a", "b"])
def test_ssim_exact_restatement(oracle, tag):
    """The float64 SSIM maps (the GPU SSIM parity bar's anchor) against the reference's golden value and the float32
    restatement."""
    a = _load("golden_ssim.npz")
    img1, img2 = a[f"{tag}_img1"], a[f"{tag}_img2"]
    ref = O.ssim_forward(img1, img2)
    ex = O.ssim_forward_exact(img1, img2)
    assert abs(float(ex[0].mean()) - float(a[f"{tag}_value"])) < 2e-6
    for r, e in zip(ref, ex):
        assert np.abs(r - e).max() <= 1e-5 * max(1.0, np.abs(e).max())
    dmap = np.full_like(ref[0], 1.0 / ref[0].size)
    g, ge = O.ssim_backward(img1, img2, dmap, *ref[1:]), O.ssim_backward_exact(img1, img2, dmap, *ref[1:])
    assert np.abs(g - ge).max() <= 1e-5 * np.abs(ge).max()


@pytest.mark.parametrize("name", ["golden_raster_64x48.npz", "golden_raster_133x97_aa.npz"])
def test_oracle_raster_regression(oracle, name):
    a = _load(name)
    col, radii, invd, st = _forward(a, int(a["deg"]), bg=a["bg"], aa=bool(a["antialiasing"]))
    assert st.num_rendered == int(a["num_rendered"])
    assert st.num_valid == int(a["num_instances"])
    np.testing.assert_array_equal(radii, a["radii"])
    t, g, _ = st.sorted_list()
    np.testing.assert_array_equal(t, a["tiles"])
    np.testing.assert_array_equal(g, a["gids"])
    np.testing.assert_array_equal(st.ranges(), a["ranges"])
    np.testing.assert_allclose(col, a["color"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(invd, a["invdepth"], rtol=0, atol=1e-6)
    go = st.backward(a["grad_color"], a["grad_invdepth"])
    for k, v in go.items():
        ref = a["g_" + k]
        tol = 1e-6 * max(1.0, float(np.abs(ref).max()))
        np.testing.assert_allclose(v, ref, rtol=0, atol=tol, err_msg=k)
