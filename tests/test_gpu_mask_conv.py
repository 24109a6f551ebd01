"""The appearance embedding's kernels (masks.py:8-54, the geometry.mask of mipnerf360.yaml / urban3d_admm.yaml;
DESIGN.md §3): dg_conv3x3 (its 3x3 convolutions' forward and input gradient) and dg_conv3x3_wgrad (weight / bias
gradient) -- MIOpen's calls replaced -- and dg_mask_head_*, its full-resolution head (resize -> conv 16 -> 8 -> ReLU ->
conv 8 -> 3) fused.

* against a float64 reference (nine shifted float64 GEMMs on the device) at the embedding's real shapes -- the
  full-resolution 16 -> 8 and 8 -> 3 convolutions at 1920 x 1080, the upsampling stages 8 -> 16 at 544 x 960, 16 -> 32 at
  272 x 480, 32 -> 64 at 136 x 240 -- and at ragged ones (1 x 1 images, widths and heights off the 64 x TR tiles):
  norm-wise relative error < 1e-5 (the fp32 sums of 2M products), and within 1e-4 of MIOpen's fp32 result;
* deterministic: two calls are bit-identical;
* dg_conv3x3's forward and adjoint against float64 at the same shapes, 1e-5;
* the head against torch's float64 resize + convolutions with autograd, up- and downsampling and ragged sizes, 1e-5;
  its backward bitwise repeatable;
* the module: AppearanceEmbedding's mask and gradients (fused head, Conv3x3) against the same network through torch's
  own ops within 1e-5 / 1e-4, and bitwise repeatable.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [(16, 8, 1080, 1920), (8, 3, 1080, 1920), (8, 16, 544, 960), (16, 32, 272, 480), (32, 64, 136, 240),
          (67, 256, 34, 60), (64, 128, 68, 120), (19, 33, 20, 70),
          (3, 5, 17, 70), (1, 1, 1, 1), (7, 9, 33, 65), (2, 3, 5, 129)]


def _wgrad(x, g, gate=None, shuffle=False):
    from dogs_amd import _lib
    L = _lib.load()
    cin, H, W = x.shape
    if shuffle:
        cin, H, W = cin // 4, 2 * H, 2 * W
    cout = g.shape[0]
    dw = torch.empty((cout, cin, 3, 3), dtype=torch.float32, device=x.device)
    db = torch.empty(cout, dtype=torch.float32, device=x.device)
    n = int(L.dg_conv3x3_wgrad_scratch_bytes(cin, cout, H, W))
    s = torch.empty(max(n, 1), dtype=torch.uint8, device=x.device)
    _lib.check(L.dg_conv3x3_wgrad(cin, cout, H, W, x.data_ptr(), g.data_ptr(),
                                  gate.data_ptr() if gate is not None else None, 4 if shuffle else 0,
                                  dw.data_ptr(), db.data_ptr(),
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
    assert L.dg_conv3x3_wgrad(5000, 2, 8, 8, 1, 1, None, 0, 1, 1, 1, 1 << 30, None) != 0
    assert L.dg_conv3x3_wgrad(2, 2, 8, 8, 1, 1, None, 1, 1, 1, 1, 1 << 30, None) != 0   # unknown flag
    assert L.dg_conv3x3_wgrad(2, 2, 8, 9, 1, 1, None, 4, 1, 1, 1, 1 << 30, None) != 0   # odd size with the shuffle
    assert L.dg_conv3x3(0, 2, 8, 8, 1, 1, None, 1, 0, None, None) != 0
    assert L.dg_conv3x3(2, 2, 8, 8, 1, 1, None, 1, 8, None, None) != 0   # unknown flag
    assert L.dg_conv3x3(2, 2, 7, 8, 1, 1, None, 1, 4, None, None) != 0   # odd size with the shuffle


def _conv(x, w, b, adjoint, relu=False, gate=None):
    from dogs_amd import _lib
    L = _lib.load()
    cout, cin = w.shape[:2]
    _, H, W = x.shape
    y = torch.full(((cin if adjoint else cout), H, W), float("nan"), device=x.device)
    flags = (1 if adjoint else 0) | (2 if relu else 0)
    _lib.check(L.dg_conv3x3(cin, cout, H, W, x.data_ptr(), w.data_ptr(), b.data_ptr() if b is not None else None,
                            y.data_ptr(), flags, gate.data_ptr() if gate is not None else None,
                            _lib.stream_of(x.device)))
    return y


def _conv64(x, w, b, adjoint):
    """float64 shifted GEMMs: the forward y = b + sum_k W_k X_k, or the input gradient of dy = x."""
    cout, cin = w.shape[:2]
    _, H, W = x.shape
    wd, xd = w.double(), x.double()
    if not adjoint:
        xp = F.pad(xd, (1, 1, 1, 1))
        y = torch.zeros((cout, H * W), dtype=torch.float64, device=x.device)
        for ky in range(3):
            for kx in range(3):
                y += wd[:, :, ky, kx] @ xp[:, ky:ky + H, kx:kx + W].reshape(cin, -1)
        if b is not None:
            y += b.double()[:, None]
        return y.reshape(cout, H, W)
    dxp = torch.zeros((cin, H + 2, W + 2), dtype=torch.float64, device=x.device)
    g = xd.reshape(cout, -1)
    for ky in range(3):
        for kx in range(3):
            dxp[:, ky:ky + H, kx:kx + W] += (wd[:, :, ky, kx].T @ g).reshape(cin, H, W)
    return dxp[:, 1:H + 1, 1:W + 1]


@pytest.mark.parametrize("cin,cout,H,W", SHAPES + [(256, 67, 34, 60), (3, 67, 9, 64), (8, 24, 40, 130)])
def test_conv_and_its_adjoint_match_float64(hip_device, cin, cout, H, W):
    """dg_conv3x3's forward (with and without bias) and adjoint against float64: the embedding's shapes (fusion
    67 -> 256 at 34 x 60 and its adjoint, every upsampling stage, the full-resolution convolutions when the fused head
    does not apply) and ragged ones -- 1 x 1, channel counts off the 8-channel groups (67, 33, 5, 3), rows and columns
    off the tiles.  Norm-wise 1e-5 (fp32 sums of up to 2304 products); bit-identical on a second call; every output
    written (NaN-filled before)."""
    gen = torch.Generator(device=hip_device).manual_seed(cin * 17 + cout * 5 + W)
    x = torch.randn((cin, H, W), generator=gen, device=hip_device)
    w = torch.randn((cout, cin, 3, 3), generator=gen, device=hip_device) / (3 * cin ** 0.5)
    b = torch.randn(cout, generator=gen, device=hip_device)
    g = torch.randn((cout, H, W), generator=gen, device=hip_device)
    for bias in (b, None):
        y = _conv(x, w, bias, False)
        assert torch.isfinite(y).all()
        assert _rel(y, _conv64(x, w, bias, False)) < 1e-5
        assert torch.equal(y, _conv(x, w, bias, False))
    dx = _conv(g, w, None, True)
    assert torch.isfinite(dx).all()
    assert _rel(dx, _conv64(g, w, None, True)) < 1e-5
    assert torch.equal(dx, _conv(g, w, None, True))


def _resize64(x, size):
    """Bilinear resize (align_corners=False) of x [C, h, w] in float64 arithmetic with the float32 source indices and
    weights of torch's float32 kernel (its weight matrices, read off by resizing one-hot images in float32): the
    reference the float32 routes are measured against.  (torch's float64 kernel computes the indices in float64, and
    the 1e-7 index difference, scaled by the gradients, swamped the summation error being measured.)"""
    _, h, w = x.shape
    H, W = size
    eh = torch.eye(h, device=x.device).reshape(1, h, h, 1)
    ew = torch.eye(w, device=x.device).reshape(1, w, 1, w)
    ry = F.interpolate(eh, size=(H, 1), mode="bilinear")[0, :, :, 0].T.double()    # [H, h]
    rx = F.interpolate(ew, size=(1, W), mode="bilinear")[0, :, 0, :].T.double()    # [W, w]
    return torch.einsum("yi,cij,xj->cyx", ry, x, rx)


def _torch_embedding(net, img, index, size, resize=None):
    """AppearanceEmbedding.forward through torch's own ops (nn.Conv2d / F.interpolate / F.conv2d), same parameters."""
    _, h, w = img.shape
    code = net.appearance_embedding[index]
    x = torch.cat([img, code[:, None, None].expand(code.shape[0], h, w)], dim=0)
    x = F.conv2d(x, net.fusion.weight, net.fusion.bias, padding=1)
    for st in net.upsample:
        x = F.relu(F.conv2d(F.pixel_shuffle(x[None], 2)[0], st[1].weight, st[1].bias, padding=1))
    x = resize(x, size) if resize else F.interpolate(x[None], size=size, mode="bilinear")[0]
    x = F.relu(F.conv2d(x, net.out_conv[0].weight, net.out_conv[0].bias, padding=1))
    return F.conv2d(x, net.out_conv[2].weight, net.out_conv[2].bias, padding=1)


@pytest.mark.parametrize("img_hw,size,branches", [((34, 60), (1080, 1920), "fixed"), ((34, 60), (540, 960), "fixed"),
                                                  ((2, 2), (150, 140), "fixed"), ((34, 60), (540, 960), "random")])
def test_embedding_gradients_match_torch(hip_device, img_hw, size, branches):
    """The module (fused head, Conv3x3 on dg_conv3x3 / dg_conv3x3_wgrad) against the same network in float64 (with
    float32 resize weights, _resize64) through torch's ops.  "fixed": every ReLU's biases are +-10 (channels
    alternately live and dead) and its weights scaled by 0.1, so no pre-activation lies within rounding of 0 and float32 and float64 take the same
    branches: the mask and every parameter gradient within 1e-5 norm-wise (~1e-6 measured, torch's float32 route
    alike).  "random": the reference's initialisation, where a few pre-activations sit within rounding of 0 and flip
    between any two summation orders -- both float32 routes then sit ~1e-4 from float64 (gpurun_out/cv4): within 1e-3.
    The third case upsamples more than 4x, so the head runs unfused (resize + Conv3x3)."""
    import copy
    from dogs_amd.masks import AppearanceEmbedding
    torch.manual_seed(3)
    net = AppearanceEmbedding(4).to(hip_device)
    with torch.no_grad():
        net.appearance_embedding.normal_(0.0, 0.3)
        if branches == "fixed":
            for conv in [st[1] for st in net.upsample] + [net.out_conv[0]]:
                conv.weight.mul_(0.1)   # pre-activations 10 +- 1.5 (min |pre| 8.97 in float64 at these inputs)
                conv.bias.copy_(torch.tensor([10.0, -10.0], device=hip_device).repeat(conv.out_channels // 2))
    net64 = copy.deepcopy(net).double()
    img = torch.rand((3,) + img_hw, device=hip_device)
    g = torch.randn((3,) + size, generator=torch.Generator(device=hip_device).manual_seed(9), device=hip_device)
    outs = []
    for route in ("module", "torch", "float64"):
        m = net64 if route == "float64" else net
        m.zero_grad(set_to_none=True)
        if route == "module":
            y = net(img, 2, size)
        else:
            y = _torch_embedding(m, img.double() if route == "float64" else img, 2, size,
                                 _resize64 if route == "float64" else None)
        (y * (g.double() if route == "float64" else g)).sum().backward()
        outs.append((y.detach(), {k: p.grad.clone() for k, p in m.named_parameters()}))
    (y0, g0), (y1, g1), (y64, g64) = outs
    bar = 1e-5 if branches == "fixed" else 1e-3
    assert _rel(y0, y64) < bar, (_rel(y0, y64), _rel(y1, y64))
    for k in g0:
        e0, e1 = _rel(g0[k], g64[k]), _rel(g1[k], g64[k])
        print(f"{k}: module {e0:.3g}, torch fp32 {e1:.3g} from float64")
        assert e0 < bar, (k, e0, e1)
    # bitwise repeatable (the ADMM ranks and the sequential baseline rely on it): every parameter's gradient again
    net.zero_grad(set_to_none=True)
    (net(img, 2, size) * g).sum().backward()
    for k, p in net.named_parameters():
        assert torch.equal(p.grad, g0[k]), k


def _head(u, w1, b1, w2, b2, size):
    from dogs_amd.masks import _MaskHead
    return _MaskHead.apply(u, w1, b1, w2, b2, size)


def _head64(u, w1, b1, w2, b2, size):
    x = _resize64(u.double(), size)
    h = F.relu(F.conv2d(x, w1.double(), b1.double(), padding=1))
    return F.conv2d(h, w2.double(), b2.double(), padding=1)


@pytest.mark.parametrize("uh,uw,H,W", [(544, 960, 1080, 1920), (48, 80, 77, 131), (544, 960, 540, 960),
                                       (544, 960, 270, 480), (3, 5, 9, 17)])
def test_mask_head_matches_float64(hip_device, uh, uw, H, W):
    """dg_mask_head_forward / _backward (resize -> conv 16 -> 8 -> ReLU -> conv 8 -> 3) against float64 resize (with
    torch's float32 source indices and weights, which this kernel computes the same way: _resize64) and convolutions
    with autograd: the mask and every gradient within 1e-5 norm-wise; the backward bitwise repeatable.  The hidden
    biases put every pre-activation of
    channels 0-5 far above 0 and of 6-7 far below it, so fp32 and fp64 take the same ReLU branch everywhere (a
    pre-activation within rounding of 0 flips between any two summation orders) and both branches are checked."""
    gen = torch.Generator(device=hip_device).manual_seed(uh + W)
    u = torch.relu(torch.randn((16, uh, uw), generator=gen, device=hip_device))
    w1 = torch.randn((8, 16, 3, 3), generator=gen, device=hip_device) * 0.1
    b1 = torch.tensor([5.0] * 6 + [-5.0] * 2, device=hip_device)
    w2 = torch.randn((3, 8, 3, 3), generator=gen, device=hip_device) * 0.1
    b2 = torch.randn(3, generator=gen, device=hip_device) * 0.1
    dm = torch.randn((3, H, W), generator=gen, device=hip_device)
    leaves = [t.clone().requires_grad_(True) for t in (u, w1, b1, w2, b2)]
    m = _head(*leaves, (H, W))
    m.backward(dm)
    got = [t.grad.clone() for t in leaves]
    ref = [t.clone().double().requires_grad_(True) for t in (u, w1, b1, w2, b2)]
    m64 = _head64(*ref, (H, W))
    m64.backward(dm.double())
    assert _rel(m, m64) < 1e-5, _rel(m, m64)
    for name, a, b in zip(("du", "dw1", "db1", "dw2", "db2"), got, ref):
        if name == "db1":     # channels 6-7 are dead: their bias gradient is exactly 0 on both
            assert torch.equal(a[6:], torch.zeros_like(a[6:])) and float(b.grad[6:].abs().max()) == 0.0
            a, b = a[:6], b.grad[:6]
        else:
            b = b.grad
        assert _rel(a, b) < 1e-5, (name, _rel(a, b))
    for t in leaves:
        t.grad = None
    _head(*leaves, (H, W)).backward(dm)
    for a, t in zip(got, leaves):
        assert torch.equal(a, t.grad)


def test_embedding_bitwise_across_processes(hip_device, tmp_path):
    """The embedding's mask and every parameter gradient are the same bits in other processes (two fresh children
    running concurrently on the same GPU) as in this one, after this process has run MIOpen convolutions of its own.
    With MIOpen inside the embedding this failed: the algorithm MIOpen picks depends on its find database and on what
    ran before in the process, and the masked ADMM ranks stopped matching the sequential baseline (gpurun_out/det1)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    probe = os.path.join(root, "tools", "embed_det_probe.py")
    sys.path.insert(0, os.path.join(root, "tools"))
    try:
        import embed_det_probe
    finally:
        sys.path.pop(0)
    x = torch.randn((1, 67, 34, 60), device=hip_device, requires_grad=True)
    w = torch.randn((256, 67, 3, 3), device=hip_device, requires_grad=True)
    F.conv2d(x, w, padding=1).square().sum().backward()     # MIOpen state in this process
    torch.cuda.synchronize()
    paths = [str(tmp_path / f"child{i}.pt") for i in range(2)]
    procs = [subprocess.Popen([sys.executable, probe, "--child", p, "--W", "960", "--H", "540"]) for p in paths]
    mine = embed_det_probe.once(960, 540)
    for p in procs:
        assert p.wait(timeout=240) == 0
    for p in paths:
        other = torch.load(p, weights_only=True)
        assert sorted(other) == sorted(mine)
        for k in mine:
            assert torch.equal(mine[k], other[k]), k


def test_mask_head_backward_same_bits_with_stored_hidden(hip_device):
    """The backward with the forward's stored hidden layer (the default: k_head_bwd_h skips the samples and conv1) and
    with it recomputed (hidden = NULL) give the same bits: the forward stores exactly the values the recomputation
    produces (one conv1 function, the same summation order)."""
    from dogs_amd import _lib
    L = _lib.load()
    gen = torch.Generator(device=hip_device).manual_seed(21)
    H, W, h2, w2 = 77, 131, 48, 80
    u = torch.relu(torch.randn((16, h2, w2), generator=gen, device=hip_device))
    w1 = torch.randn((8, 16, 3, 3), generator=gen, device=hip_device) * 0.1
    b1 = torch.randn(8, generator=gen, device=hip_device) * 0.1
    w2_ = torch.randn((3, 8, 3, 3), generator=gen, device=hip_device) * 0.1
    b2 = torch.randn(3, generator=gen, device=hip_device) * 0.1
    dm = torch.randn((3, H, W), generator=gen, device=hip_device)
    P = [t.data_ptr() for t in (u, w1, b1, w2_, b2)]
    st = _lib.stream_of(hip_device)
    mask = torch.empty((3, H, W), device=hip_device)
    hid = torch.full((8, H, W), float("nan"), device=hip_device)
    _lib.check(L.dg_mask_head_forward(H, W, h2, w2, *P, mask.data_ptr(), hid.data_ptr(), st))
    mask2 = torch.empty_like(mask)
    _lib.check(L.dg_mask_head_forward(H, W, h2, w2, *P, mask2.data_ptr(), None, st))
    assert torch.equal(mask, mask2) and torch.isfinite(hid).all() and (hid >= 0).all()
    nb = int(L.dg_mask_head_scratch_bytes(H, W))
    outs = []
    for h in (hid.data_ptr(), None):
        du = torch.empty_like(u)
        dp = torch.empty(int(L.dg_mask_head_nparams()), device=hip_device)
        scr = torch.empty(nb, dtype=torch.uint8, device=hip_device)
        _lib.check(L.dg_mask_head_backward(H, W, h2, w2, *P, dm.data_ptr(), h, du.data_ptr(), dp.data_ptr(),
                                           scr.data_ptr(), nb, st))
        outs.append((du, dp))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_conv3x3_module_batched_and_unbatched(hip_device):
    """Conv3x3 (the embedding's nn.Conv2d on dg_conv3x3 / dg_conv3x3_wgrad) on a batch of 2 and on one unbatched
    image: output and the input / weight / bias gradients against float64 autograd of F.conv2d, 1e-5 norm-wise (the
    weight gradient summed over the batch in batch order)."""
    from dogs_amd.masks import Conv3x3
    torch.manual_seed(4)
    conv = Conv3x3(5, 7).to(hip_device)
    for shape in ((2, 5, 9, 13), (5, 17, 70)):
        x = torch.randn(shape, device=hip_device, requires_grad=True)
        g = torch.randn(((shape[0],) if len(shape) == 4 else ()) + (7,) + shape[-2:], device=hip_device)
        conv.zero_grad(set_to_none=True)
        y = conv(x)
        (y * g).sum().backward()
        x64 = x.detach().double().requires_grad_(True)
        w64 = conv.weight.detach().double().requires_grad_(True)
        b64 = conv.bias.detach().double().requires_grad_(True)
        y64 = F.conv2d(x64, w64, b64, padding=1)
        (y64 * g.double()).sum().backward()
        assert y.shape == y64.shape
        assert _rel(y, y64) < 1e-5
        assert _rel(x.grad, x64.grad) < 1e-5
        assert _rel(conv.weight.grad, w64.grad) < 1e-5 and _rel(conv.bias.grad, b64.grad) < 1e-5


@pytest.mark.parametrize("cin,cout,H,W", [(8, 16, 544, 960), (64, 128, 68, 120), (7, 9, 33, 65)])
def test_relu_folded_into_conv_and_its_backward(hip_device, cin, cout, H, W):
    """The stages' ReLU folded into the kernels: the forward with DG_CONV_RELU = max(conv, 0) of the plain forward (bit
    for bit: the same sums, then the clamp); the adjoint and the weight gradient with gate = that output equal the
    plain kernels applied to dy * [y > 0] (bit for bit), and float64 within 1e-5."""
    gen = torch.Generator(device=hip_device).manual_seed(cin + cout + W)
    x = torch.randn((cin, H, W), generator=gen, device=hip_device)
    w = torch.randn((cout, cin, 3, 3), generator=gen, device=hip_device) / (3 * cin ** 0.5)
    b = torch.randn(cout, generator=gen, device=hip_device) * 0.3
    g = torch.randn((cout, H, W), generator=gen, device=hip_device)
    y = _conv(x, w, b, False, relu=True)
    plain = _conv(x, w, b, False)
    assert torch.equal(y, torch.clamp_min(plain, 0.0)) and 0.1 < float((y > 0).float().mean()) < 0.9
    gm = torch.where(y > 0, g, torch.zeros_like(g))
    assert torch.equal(_conv(g, w, None, True, gate=y), _conv(gm, w, None, True))
    dw, db = _wgrad(x, g, gate=y)
    dw2, db2 = _wgrad(x, gm)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)
    rw, rb = _ref64(x, gm)
    assert _rel(dw, rw) < 1e-5 and _rel(db, rb) < 1e-5
    assert _rel(_conv(g, w, None, True, gate=y), _conv64(gm, w, None, True)) < 1e-5


@pytest.mark.parametrize("cin,cout,H,W", [(16, 32, 272, 480), (64, 128, 68, 120), (3, 5, 34, 130)])
def test_pixel_shuffle_folded_into_conv_and_its_backward(hip_device, cin, cout, H, W):
    """The stages' PixelShuffle(2) folded into the kernels' addressing (DG_CONV_SHUFFLE): the forward of xq [4 cin][H/2]
    [W/2] equals the plain forward of pixel_shuffle(xq) bit for bit (the same sums over the same values), the adjoint
    equals pixel_unshuffle of the plain adjoint and the weight gradient the plain one of the shuffled input, both bit
    for bit, with and without the ReLU gate; the Conv3x3 module with shuffle=True equals float64 within 1e-5."""
    gen = torch.Generator(device=hip_device).manual_seed(cin * 3 + cout + W)
    xq = torch.randn((4 * cin, H // 2, W // 2), generator=gen, device=hip_device)
    x = F.pixel_shuffle(xq[None], 2)[0].contiguous()
    w = torch.randn((cout, cin, 3, 3), generator=gen, device=hip_device) / (3 * cin ** 0.5)
    b = torch.randn(cout, generator=gen, device=hip_device) * 0.3
    g = torch.randn((cout, H, W), generator=gen, device=hip_device)
    from dogs_amd import _lib
    L = _lib.load()
    st = _lib.stream_of(x.device)
    for relu in (False, True):
        ys = torch.full((cout, H, W), float("nan"), device=hip_device)
        _lib.check(L.dg_conv3x3(cin, cout, H, W, xq.data_ptr(), w.data_ptr(), b.data_ptr(), ys.data_ptr(),
                                4 | (2 if relu else 0), None, st))
        y = _conv(x, w, b, False, relu=relu)
        assert torch.equal(ys, y)
        gate = y if relu else None
        dq = torch.full((4 * cin, H // 2, W // 2), float("nan"), device=hip_device)
        _lib.check(L.dg_conv3x3(cin, cout, H, W, g.data_ptr(), w.data_ptr(), None, dq.data_ptr(), 5,
                                gate.data_ptr() if relu else None, st))
        assert torch.equal(dq, F.pixel_unshuffle(_conv(g, w, None, True, gate=gate)[None], 2)[0])
        dws, dbs = _wgrad(xq, g, gate=gate, shuffle=True)
        dw, db = _wgrad(x, g, gate=gate)
        assert torch.equal(dws, dw) and torch.equal(dbs, db)
    from dogs_amd.masks import Conv3x3
    conv = Conv3x3(cin, cout).to(hip_device)
    xr = xq[None].clone().requires_grad_(True)
    y = conv(xr, relu=True, shuffle=True)
    (y * g).sum().backward()
    x64 = xq[None].double().requires_grad_(True)
    w64 = conv.weight.detach().double().requires_grad_(True)
    b64 = conv.bias.detach().double().requires_grad_(True)
    y64 = F.conv2d(F.pixel_shuffle(x64, 2), w64, b64, padding=1)
    # the ReLU's mask taken from the float32 output: a float64 one flips where y rounds across 0
    (y64 * torch.where(y[0] > 0, g, torch.zeros_like(g)).double()).sum().backward()
    assert _rel(y, F.relu(y64)) < 1e-5 and _rel(xr.grad, x64.grad) < 1e-5
    assert _rel(conv.weight.grad, w64.grad) < 1e-5 and _rel(conv.bias.grad, b64.grad) < 1e-5
