"""dg_conv3x3_wgrad: the weight / bias gradient of the appearance embedding's 3x3 convolutions (masks.py:8-54, the
geometry.mask of mipnerf360.yaml / urban3d_admm.yaml), replacing MIOpen's backward-weights call.

* against a float64 reference (nine shifted float64 GEMMs on the device) at the embedding's real shapes -- the
  full-resolution 16 -> 8 and 8 -> 3 convolutions at 1920 x 1080, the upsampling stages 8 -> 16 at 544 x 960, 16 -> 32 at
  272 x 480, 32 -> 64 at 136 x 240 -- and at ragged ones (1 x 1 images, widths and heights off the 64 x TR tiles):
  norm-wise relative error < 1e-5 (the fp32 sums of 2M products), and within 1e-4 of MIOpen's fp32 result;
* deterministic: two calls are bit-identical;
* the module: AppearanceEmbedding's gradients through Conv3x3 equal those through plain nn.Conv2d (MIOpen) within
  1e-4, the forward bit for bit; unsupported channel counts (fusion 67 -> 256) keep MIOpen's path.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [(16, 8, 1080, 1920), (8, 3, 1080, 1920), (8, 16, 544, 960), (16, 32, 272, 480), (32, 64, 136, 240),
          (3, 5, 17, 70), (1, 1, 1, 1), (7, 9, 33, 65), (2, 3, 5, 129)]


def _wgrad(x, g):
    from dogs_amd import _lib
    L = _lib.load()
    cin, H, W = x.shape
    cout = g.shape[0]
    dw = torch.empty((cout, cin, 3, 3), dtype=torch.float32, device=x.device)
    db = torch.empty(cout, dtype=torch.float32, device=x.device)
    n = int(L.dg_conv3x3_wgrad_scratch_bytes(cin, cout, H, W))
    s = torch.empty(max(n, 1), dtype=torch.uint8, device=x.device)
    _lib.check(L.dg_conv3x3_wgrad(cin, cout, H, W, x.data_ptr(), g.data_ptr(), dw.data_ptr(), db.data_ptr(),
                                  s.data_ptr(), n, _lib.stream_of(x.device)))
    return dw, db


def _ref64(x, g):
    cin, H, W = x.shape
    cout = g.shape[0]
    xp = F.pad(x.double(), (1, 1, 1, 1))
    gd = g.double().reshape(cout, -1)
    dw = torch.empty((cout, cin, 3, 3), dtype=torch.float64, device=x.device)
    for ky in range(3):
        for kx in range(3):
            dw[:, :, ky, kx] = gd @ xp[:, ky:ky + H, kx:kx + W].reshape(cin, -1).T
    return dw, gd.sum(1)


def _rel(a, b):
    return float((a.double() - b.double()).norm() / max(float(b.double().norm()), 1e-300))


@pytest.mark.parametrize("cin,cout,H,W", SHAPES)
def test_wgrad_matches_float64(hip_device, cin, cout, H, W):
    gen = torch.Generator(device=hip_device).manual_seed(cin * 131 + cout * 7 + H)
    x = torch.randn((cin, H, W), generator=gen, device=hip_device)
    g = torch.randn((cout, H, W), generator=gen, device=hip_device)
    dw, db = _wgrad(x, g)
    rw, rb = _ref64(x, g)
    assert _rel(dw, rw) < 1e-5, _rel(dw, rw)
    assert _rel(db, rb) < 1e-5, _rel(db, rb)
    dw2, db2 = _wgrad(x, g)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)
    if H * W > 1:   # MIOpen's fp32 weight gradient of the same convolution
        w = torch.zeros((cout, cin, 3, 3), device=hip_device)
        mw = torch.ops.aten.convolution_backward(g[None], x[None], w, [cout], [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                                 [False, True, True])
        assert _rel(dw, mw[1]) < 1e-4 and _rel(db, mw[2]) < 1e-4


def test_unsupported_channels_are_an_error(hip_device):
    from dogs_amd import _lib
    L = _lib.load()
    assert L.dg_conv3x3_wgrad(67, 256, 8, 8, 1, 1, 1, 1, 1, 1 << 30, None) != 0


def test_embedding_gradients_match_miopen(hip_device):
    import copy
    from dogs_amd.masks import AppearanceEmbedding, Conv3x3
    torch.manual_seed(3)
    net = AppearanceEmbedding(4).to(hip_device)
    with torch.no_grad():
        net.appearance_embedding.normal_(0.0, 0.3)
    ref = copy.deepcopy(net)
    for name, mod in list(ref.named_modules()):   # the same parameters through plain nn.Conv2d
        for cname, child in list(mod.named_children()):
            if isinstance(child, Conv3x3):
                plain = torch.nn.Conv2d(child.in_channels, child.out_channels, 3, padding=1).to(hip_device)
                plain.load_state_dict(child.state_dict())
                setattr(mod, cname, plain)
    img = torch.rand((3, 34, 60), device=hip_device)
    g = torch.randn((3, 1080, 1920), generator=torch.Generator(device=hip_device).manual_seed(9), device=hip_device)
    outs = []
    for m in (net, ref):
        y = m(img, 2, (1080, 1920))
        (y * g).sum().backward()
        outs.append((y.detach(), {k: p.grad.clone() for k, p in m.named_parameters()}))
    (y0, g0), (y1, g1) = outs
    assert torch.equal(y0, y1)
    for k in g0:
        assert _rel(g0[k], g1[k]) < 1e-4, (k, _rel(g0[k], g1[k]))
