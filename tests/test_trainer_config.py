"""CPU checks of the trainer options the reference configs switch on (no GPU):

* GSTrainConfig.from_reference / ADMMRunConfig.from_reference read urban3d_admm.yaml and mipnerf360.yaml key for key
  (the parsed configs are committed as data, tests/golden/reference_configs.json, made by
  tests/golden/make_trainer_golden.py; when /root/reference is present the YAML files themselves are read too);
* dogs_amd.masks.AppearanceEmbedding has the reference module's state-dict keys and shapes and, with the same
  parameters, returns the reference module's mask (tests/golden/appearance_embedding.npz, produced by the reference's
  own masks.py);
* the camera-radius quirk of compute_nerf_plus_plus_norm and Camera.downsample's image size.
"""
import json
import math
import os

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
REF_CFG = "/root/reference/config/gaussian_splatting"

# (YAML path, GSTrainConfig attribute)
GS_KEYS = [
    ("trainer.max_iterations", "max_iterations"), ("geometry.densify_start_iter", "densify_start_iter"),
    ("geometry.densify_end_iter", "densify_end_iter"), ("geometry.densification_interval", "densification_interval"),
    ("geometry.opacity_reset_interval", "opacity_reset_interval"),
    ("geometry.densify_grad_threshold", "densify_grad_threshold"), ("geometry.percent_dense", "percent_dense"),
    ("geometry.depth_threshold", "depth_threshold"), ("geometry.mask", "mask"),
    ("geometry.coarse-to-fine", "coarse_to_fine"), ("prune.iterations", "prune_iterations"),
    ("prune.v_pow", "prune_v_pow"), ("prune.prune_decay", "prune_decay"), ("prune.prune_percent", "prune_percent"),
    ("optimizer.lr.position_init", "position_init"), ("optimizer.lr.position_final", "position_final"),
    ("optimizer.lr.position_delay_mult", "position_delay_mult"),
    ("optimizer.lr.position_max_iterations", "position_max_iterations"),
    ("optimizer.lr.exposure_lr_init", "exposure_lr_init"), ("optimizer.lr.exposure_lr_final", "exposure_lr_final"),
    ("optimizer.lr.exposure_lr_delay_steps", "exposure_lr_delay_steps"),
    ("optimizer.lr.exposure_lr_delay_mult", "exposure_lr_delay_mult"),
    ("optimizer.lr.exposure_max_iterations", "exposure_max_iterations"),
    ("optimizer.lr.feature", "feature"), ("optimizer.lr.opacity", "opacity"), ("optimizer.lr.scaling", "scaling"),
    ("optimizer.lr.quaternion", "quaternion"), ("optimizer.lr.mask", "mask_lr"),
    ("texture.max_sh_degree", "max_sh_degree"), ("texture.anti_aliasing", "anti_aliasing"),
    ("appearance.use_trained_exposure", "use_trained_exposure"), ("loss.lambda_dssim", "lambda_dssim"),
    ("loss.lambda_scale", "lambda_scale"), ("loss.lambda_mask", "lambda_mask"),
    ("dataset.apply_mask", "white_background"),
]
ADMM_KEYS = ["consensus_interval", "alpha_xyz", "alpha_fdc", "alpha_fr", "alpha_s", "alpha_q", "alpha_o",
             "stop_adapt_iter", "mu", "tau_inc", "tau_dec", "over_relaxation_coeff"]


def _get(d, path):
    for p in path.split("."):
        d = d[p]
    return d


def _resolved(d, v):
    if isinstance(v, str) and v.startswith("${"):
        return _resolved(d, _get(d, v[2:-1]))
    return v


def _sources():
    with open(os.path.join(GOLD, "reference_configs.json"), encoding="utf-8") as f:
        fixed = json.load(f)
    out = [(name, d) for name, d in sorted(fixed.items())]
    if os.path.isdir(REF_CFG):
        out += [(name, os.path.join(REF_CFG, name)) for name in sorted(fixed)]
    return out


@pytest.mark.parametrize("name,src", _sources(), ids=lambda x: x if isinstance(x, str) and len(x) < 40 else "")
def test_config_from_reference_key_for_key(name, src):
    from dogs_amd.admm_run import ADMMRunConfig
    from dogs_amd.trainer import GSTrainConfig, load_reference_config
    d = load_reference_config(src)
    c = GSTrainConfig.from_reference(src)
    for path, attr in GS_KEYS:
        want = _resolved(d, _get(d, path))
        got = getattr(c, attr)
        if isinstance(want, list):
            assert tuple(got) == tuple(want), (path, got, want)
        elif isinstance(want, bool):
            assert got is want, (path, got, want)
        else:
            assert got == pytest.approx(float(want), rel=0, abs=0), (path, got, want)
    # absent keys: spatial_lr_scale computed from the cameras (-1), no prune iterations when the list is empty
    assert c.spatial_lr_scale == float(d["geometry"].get("spatial_lr_scale", -1))
    if name == "urban3d_admm.yaml":
        assert (c.mask, c.lambda_mask, c.depth_threshold, c.mask_lr) == (True, 0.5, 0.23, 0.001)
        assert c.prune_iterations == (29800,) and c.lambda_scale == 0.05 and c.position_max_iterations == 30000
        r = ADMMRunConfig.from_reference(src)
        a = d["trainer"]["admm"]
        for k in ADMM_KEYS:
            assert getattr(r.admm, k) == pytest.approx(float(a[k]), rel=0, abs=0), k
        assert r.admm.consensus_interval == 200 and r.admm.stop_adapt_iter == 32000
        assert r.gs == c
    else:   # mipnerf360 (BASELINE config 2): the mask is on with lambda_mask 0
        assert (c.mask, c.lambda_mask, c.depth_threshold) == (True, 0.0, 0.0)
        assert c.position_max_iterations == c.max_iterations == 30000


def _fill(key, shape):
    n = int(np.prod(shape)) if len(shape) else 1
    h = sum(ord(ch) for ch in key) % 97
    x = torch.arange(n, dtype=torch.float64)
    v = 0.05 * torch.sin(0.37 * x + h) + 0.01 * torch.cos(0.011 * x * (1 + h % 5))
    return v.reshape(shape).to(torch.float32)


def test_appearance_embedding_matches_reference_module():
    from dogs_amd.masks import AppearanceEmbedding
    g = np.load(os.path.join(GOLD, "appearance_embedding.npz"))
    net = AppearanceEmbedding(5)
    sd = net.state_dict()
    assert sorted(sd) == list(g["keys"])
    for k, s in zip(g["keys"], g["shapes"]):
        assert list(sd[k].shape) == json.loads(str(s)), k
    net.load_state_dict({k: _fill(k, tuple(v.shape)) for k, v in sd.items()})
    torch.set_num_threads(1)
    with torch.no_grad():
        out = net(torch.from_numpy(g["image"]), 2, (100, 130))
    assert out.shape == (3, 100, 130)
    np.testing.assert_allclose(out.numpy(), g["out"], rtol=0, atol=1e-6)


def test_nerf_plus_plus_norm_reference_quirk():
    """Camera centres as [1, 3] rows hstacked to [1, 3n]: the mean of all coordinates, max |coordinate - mean|."""
    from dogs_amd.camera import make_camera
    from dogs_amd.trainer import nerf_plus_plus_norm
    rng = np.random.default_rng(2)
    cams = []
    for _ in range(7):
        w2c = torch.eye(4)
        w2c[:3, 3] = torch.from_numpy(rng.normal(size=3)).float() * 3
        cams.append(make_camera(64, 48, 50.0, 50.0, world_to_camera=w2c))
    c = np.concatenate([cam.camera_center.numpy().reshape(-1) for cam in cams])
    assert nerf_plus_plus_norm(cams) == pytest.approx(1.1 * float(np.max(np.abs(c - c.mean()))), rel=1e-6)


def test_downsample_sizes_and_camera():
    from dogs_amd.camera import make_camera
    from dogs_amd.masks import downsample_image
    img = torch.rand(3, 1080, 1917)
    assert downsample_image(img, 32).shape == (3, math.ceil(1080 / 32), math.ceil(1917 / 32))
    assert downsample_image(img, 1) is img
    cam = make_camera(1917, 1080, 1600.0, 1500.0, image_index=7)
    d = cam.downsample(4)
    assert (d.width, d.height, d.image_index) == (480, 270, 7)
    assert math.tan(d.fov_x / 2) == pytest.approx(480 / (2 * 400.0), rel=1e-9)
    assert math.tan(d.fov_y / 2) == pytest.approx(270 / (2 * 375.0), rel=1e-9)
    torch.testing.assert_close(d.camera_center, cam.camera_center)
