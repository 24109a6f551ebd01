"""Fused parameter activations (dogs_amd.activations, optim.hip k_activate_*) against the plain PyTorch fp32 ops the
reference's GaussianSplatModel uses (sigmoid, exp, F.normalize): values bit for bit (the quaternion norm summed
pairwise as torch's vector_norm sums it; tools/act_match_probe.py), gradients within 2e-6 relative (the normalize
backward is one fused expression here, a chain of torch ops there; the tolerance is written below), zero-norm rotations
included."""
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
        assert torch.equal(x, y)
    w = [torch.randn(t.shape, generator=g).to(hip_device) for t in (o, s, q)]
    sum((x * y).sum() for x, y in zip((o, s, q), w)).backward()
    sum((x * y).sum() for x, y in zip((o2, s2, q2), w)).backward()
    for x, y in zip(a, b):
        torch.testing.assert_close(x.grad, y.grad, rtol=2e-6, atol=1e-6 * float(y.grad.abs().max()))
    # a contiguous slice that starts mid-row (not 16-B aligned) is accepted
    o3, s3, q3 = activate(ro[1:], rs[1:], rq[1:])
    torch.testing.assert_close(q3, torch.nn.functional.normalize(rq[1:]), rtol=2e-6, atol=1e-7)
    # a truly misaligned [N,4] rotation view (rows start 4 B past a 16-B boundary): the float4 path gets a copy
    mis = torch.empty(4 * n + 1, device=hip_device)[1:].view(n, 4).copy_(rq)
    assert mis.data_ptr() % 16 != 0
    mq = mis.detach().requires_grad_(True)
    assert mq.data_ptr() % 16 != 0
    rq_ref = rq.clone().requires_grad_(True)
    q4 = activate(ro, rs, mq)[2]
    q5 = torch.nn.functional.normalize(rq_ref)
    torch.testing.assert_close(q4, q5, rtol=2e-6, atol=1e-7)
    wq = torch.randn(q4.shape, generator=g).to(hip_device)
    (q4 * wq).sum().backward()
    (q5 * wq).sum().backward()
    torch.testing.assert_close(mq.grad, rq_ref.grad, rtol=2e-6, atol=1e-6 * float(rq_ref.grad.abs().max()))
    # a missing incoming gradient counts as zeros
    c = [t.clone().requires_grad_(True) for t in (ro, rs, rq)]
    activate(*c)[1].sum().backward()
    assert float(c[0].grad.abs().max()) == 0.0 and float(c[2].grad.abs().max()) == 0.0
    torch.testing.assert_close(c[1].grad, torch.exp(rs), rtol=2e-6, atol=0)


def test_activations_reject_foreign_tensors(hip_device):
    """A host tensor or a float64 parameter raises like torch's own ops instead of handing the kernel a host pointer
    or doubles read as floats."""
    from dogs_amd.activations import activate
    n = 16
    ro, rs, rq = torch.zeros(n, 1, device=hip_device), torch.zeros(n, 3, device=hip_device), torch.ones(n, 4, device=hip_device)
    with pytest.raises(RuntimeError):
        activate(ro, rs.cpu(), rq)
    with pytest.raises(RuntimeError):
        activate(ro, rs, rq.double())
    with pytest.raises(RuntimeError):
        activate(ro.cpu(), rs, rq)


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
    # NaN propagates as in torch.clamp (a diverged render must not read as a finite loss); its gradient is 0
    x = torch.tensor([[0.5, float("nan"), 1.5, -1.0, 0.25]], device=hip_device).expand(3, 5).contiguous()
    y = torch.full_like(x, 0.5)
    a = x.clone().requires_grad_(True)
    c1, l1 = clamp_l1(a, y)
    c2 = x.clamp(0, 1)
    assert torch.equal(torch.isnan(c1), torch.isnan(c2)) and bool(torch.isnan(l1))
    torch.testing.assert_close(c1[~torch.isnan(c1)], c2[~torch.isnan(c2)], rtol=0, atol=0)
    (c1 * 1.0).sum().backward()
    assert float(a.grad[0, 1]) == 0.0
    # foreign tensors raise
    with pytest.raises(RuntimeError):
        clamp_l1(img, gt.cpu())
    with pytest.raises(RuntimeError):
        clamp_l1(img, gt.double())
    flat = img.reshape(-1)[1:]                                   # misaligned start
    torch.testing.assert_close(clamp_l1(flat, gt.reshape(-1)[1:])[1], (flat.clamp(0, 1) - gt.reshape(-1)[1:]).abs().mean(),
                               rtol=1e-6, atol=0)
    # an empty image: the mean is 0 / 0 = nan, as torch's mean of an empty tensor (dg_mean_of_parts over no partials)
    e = torch.empty((3, 0, 7), device=hip_device)
    c, l1 = clamp_l1(e, e)
    assert c.shape == e.shape and bool(torch.isnan(l1)) and l1.dim() == 0


def test_fused_ssim_mean_without_train_has_no_backward(hip_device):
    """fused_ssim(..., train=False) computes the value only (no partial maps, as the reference's forward with
    train=False); a backward through it raises instead of reading absent maps."""
    from fused_ssim import fused_ssim
    g = torch.Generator().manual_seed(9)
    a = torch.rand((1, 3, 40, 60), generator=g).to(hip_device).requires_grad_(True)
    b = torch.rand((1, 3, 40, 60), generator=g).to(hip_device)
    v = fused_ssim(a, b, train=False)
    assert torch.isfinite(v)
    with pytest.raises(RuntimeError):
        v.backward()
