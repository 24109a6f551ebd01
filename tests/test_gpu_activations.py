"""Fused parameter activations (dogs_amd.activations, optim.hip k_activate_*) against the plain PyTorch fp32 ops the
reference's GaussianSplatModel uses (sigmoid, exp, F.normalize): values and gradients within 2e-6 relative
(fp32 rounding of expf / the reciprocal norm; the tolerance is written below), zero-norm rotations included."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_activations_match_torch(hip_device):
    from dogs_amd.activations import activate
    g = torch.Generator().manual_seed(0)
    n = 100_003
    ro = (torch.randn(n, 1, generator=g) * 3).to(hip_device)
    rs = (torch.randn(n, 3, generator=g) - 4).to(hip_device)
    rq = torch.randn(n, 4, generator=g).to(hip_device)
    rq[7] = 0.0                                                  # clamped denominator
    a = [t.clone().requires_grad_(True) for t in (ro, rs, rq)]
    b = [t.clone().requires_grad_(True) for t in (ro, rs, rq)]
    o, s, q = activate(*a)
    o2, s2, q2 = torch.sigmoid(b[0]), torch.exp(b[1]), torch.nn.functional.normalize(b[2])
    for x, y in ((o, o2), (s, s2), (q, q2)):
        torch.testing.assert_close(x, y, rtol=2e-6, atol=1e-7)
    w = [torch.randn(t.shape, generator=g).to(hip_device) for t in (o, s, q)]
    sum((x * y).sum() for x, y in zip((o, s, q), w)).backward()
    sum((x * y).sum() for x, y in zip((o2, s2, q2), w)).backward()
    for x, y in zip(a, b):
        torch.testing.assert_close(x.grad, y.grad, rtol=2e-6, atol=1e-6 * float(y.grad.abs().max()))
    # a contiguous slice that starts mid-row (not 16-B aligned) is accepted
    o3, s3, q3 = activate(ro[1:], rs[1:], rq[1:])
    torch.testing.assert_close(q3, torch.nn.functional.normalize(rq[1:]), rtol=2e-6, atol=1e-7)
    # a missing incoming gradient counts as zeros
    c = [t.clone().requires_grad_(True) for t in (ro, rs, rq)]
    activate(*c)[1].sum().backward()
    assert float(c[0].grad.abs().max()) == 0.0 and float(c[2].grad.abs().max()) == 0.0
    torch.testing.assert_close(c[1].grad, torch.exp(rs), rtol=2e-6, atol=0)


def test_clamp_l1_matches_torch(hip_device):
    """dogs_amd.loss.clamp_l1 vs img.clamp(0, 1) and (img - gt).abs().mean() in torch fp32: the clamped image is
    exact; the mean within 1e-6 relative (different summation order); the gradient, with an SSIM-like upstream
    gradient on the clamped image, within 1e-6 relative (exact zeros at clamp boundaries and ties)."""
    from dogs_amd.loss import clamp_l1
    g = torch.Generator().manual_seed(1)
    for shape in ((3, 1080, 1920), (3, 17, 29)):
        img = (torch.rand(shape, generator=g) * 1.4 - 0.2).to(hip_device)
        gt = torch.rand(shape, generator=g).to(hip_device)
        img.view(-1)[:5] = torch.tensor([0.0, 1.0, -0.0, 0.5, 2.0])
        gt.view(-1)[3] = 0.5                                     # a tie: sgn 0
        up = torch.randn(shape, generator=g).to(hip_device)
        a, b = img.clone().requires_grad_(True), img.clone().requires_grad_(True)
        c1, l1 = clamp_l1(a, gt)
        c2 = b.clamp(0, 1)
        l2 = (c2 - gt).abs().mean()
        assert torch.equal(c1, c2)
        torch.testing.assert_close(l1, l2, rtol=1e-6, atol=0)
        (0.8 * l1 + (c1 * up).sum() * 1e-3).backward()
        (0.8 * l2 + (c2 * up).sum() * 1e-3).backward()
        torch.testing.assert_close(a.grad, b.grad, rtol=1e-6, atol=1e-12)
    flat = img.reshape(-1)[1:]                                   # misaligned start
    torch.testing.assert_close(clamp_l1(flat, gt.reshape(-1)[1:])[1], (flat.clamp(0, 1) - gt.reshape(-1)[1:]).abs().mean(),
                               rtol=1e-6, atol=0)
