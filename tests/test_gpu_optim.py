"""GPU parity of the optimizer side of a view, through the drop-in Python surface:

* SparseGaussianAdam.step over all groups in one launch (dg_adam_update_groups) against the oracle's adam.cu
  restatement per group -- bit-exact, ragged group widths (3, 3, 45, 1, 3, 4), unaligned views (scalar path);
* the densification statistics folded into that launch (gaussian_trainer.py:433-438) -- bit-exact;
* densify_and_prune as GPU compaction (dg_densify_*) against oracle/densify_oracle.py on the same torch.normal
  split offsets: counts, row order, copied rows and Adam moments bit-exact; the split children's xyz / scaling
  within 2 ulp-scale relative error (the reference's bmm summation order is not specified)."""
import types

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

WIDTHS = {"xyz": (3,), "f_dc": (1, 3), "f_rest": (15, 3), "opacity": (1,), "scaling": (3,), "quaternion": (4,)}
LRS = {"xyz": 1.6e-4, "f_dc": 2.5e-3, "f_rest": 1.25e-4, "opacity": 2.5e-2, "scaling": 5e-3, "quaternion": 1e-3}


def _params(N, seed, dev):
    g = torch.Generator().manual_seed(seed)
    p = {k: torch.randn((N,) + s, generator=g) for k, s in WIDTHS.items()}
    p["scaling"] = torch.log(torch.rand((N, 3), generator=g) * 0.1 + 1e-3)
    p["opacity"] = torch.randn((N, 1), generator=g) * 3.0
    return {k: v.to(dev) for k, v in p.items()}, g


@pytest.mark.parametrize("N", [1, 777, 20000, 1_000_000])   # 1e6 x 59 floats: the bench / config-2 size
def test_adam_groups_and_stats_bitexact(oracle, hip_device, N):
    from diff_gaussian_rasterization import SparseGaussianAdam
    from oracle import densify_oracle as D
    params, g = _params(N, N, hip_device)
    ps = {k: torch.nn.Parameter(v.clone()) for k, v in params.items()}
    opt = SparseGaussianAdam([{"params": [ps[k]], "lr": LRS[k], "name": k} for k in ps], lr=0.0, eps=1e-15)
    vis = (torch.rand(N, generator=g) > 0.3)
    ref = {k: [v.cpu().numpy().copy(), np.zeros(v.shape, np.float32), np.zeros(v.shape, np.float32)]
           for k, v in params.items()}
    radii = (torch.rand(N, generator=g) * 30).int()
    sg = torch.randn((N, 3), generator=g)
    mr = torch.rand(N, generator=g) * 10
    acc, den = torch.rand((N, 1), generator=g), torch.randint(0, 5, (N, 1), generator=g).float()
    mr_o, acc_o, den_o = mr.numpy().copy(), acc.numpy().copy(), den.numpy().copy()
    stats = {"radii": radii.to(hip_device), "dmeans2D": sg.to(hip_device), "max_radii2D": mr.to(hip_device),
             "grad_accum": acc.to(hip_device), "denom": den.to(hip_device)}
    for it in range(2):
        grads = {k: torch.randn(v.shape, generator=g) for k, v in params.items()}
        for k in ps:
            ps[k].grad = grads[k].to(hip_device)
            r = ref[k]
            M = r[0].size // N
            oracle.adam(r[0], grads[k].numpy().copy(), r[1], r[2], vis.numpy(), LRS[k], 0.9, 0.999, 1e-15, N, M)
        opt.step(vis.to(hip_device), N, stats=stats if it == 0 else None)
    D.densification_stats(mr_o, acc_o, den_o, radii.numpy(), sg.numpy(), vis.numpy())
    for k in ps:
        st = opt.state[ps[k]]
        np.testing.assert_array_equal(ps[k].detach().cpu().numpy(), ref[k][0], err_msg=k)
        np.testing.assert_array_equal(st["exp_avg"].cpu().numpy(), ref[k][1], err_msg=k)
        np.testing.assert_array_equal(st["exp_avg_sq"].cpu().numpy(), ref[k][2], err_msg=k)
    np.testing.assert_array_equal(stats["max_radii2D"].cpu().numpy(), mr_o)
    np.testing.assert_array_equal(stats["grad_accum"].cpu().numpy(), acc_o)
    np.testing.assert_array_equal(stats["denom"].cpu().numpy(), den_o)


def test_adam_groups_unaligned_views(oracle, hip_device):
    """Groups that are views at an odd float offset take the scalar path; results stay bit-exact."""
    from diff_gaussian_rasterization import _C
    N, M = 1001, 3
    g = torch.Generator().manual_seed(5)
    base = torch.randn(4 * (N * M + 1), generator=g)
    p, gr, m, v = (base[i * (N * M + 1) + 1:(i + 1) * (N * M + 1)].view(N, M) for i in range(4))
    v.abs_()
    vis = torch.rand(N, generator=g) > 0.5
    po, mo, vo = p.numpy().copy(), m.numpy().copy(), v.numpy().copy()
    oracle.adam(po, gr.numpy().copy(), mo, vo, vis.numpy(), 1e-3, 0.9, 0.999, 1e-15, N, M)
    bd = base.to(hip_device)
    ph, gh, mh, vh = (bd[i * (N * M + 1) + 1:(i + 1) * (N * M + 1)].view(N, M) for i in range(4))
    _C.adam_update_groups([(ph, gh, mh, vh, 1e-3, 1e-15)], vis.to(hip_device), N)
    np.testing.assert_array_equal(ph.cpu().numpy(), po)
    np.testing.assert_array_equal(mh.cpu().numpy(), mo)
    np.testing.assert_array_equal(vh.cpu().numpy(), vo)


@pytest.mark.parametrize("N,bbox,screen", [(3000, None, None), (20000, (0, 0, -1.0), 20.0), (1, None, 20.0)])
def test_densify_and_prune_matches_oracle(hip_device, N, bbox, screen):
    from diff_gaussian_rasterization import SparseGaussianAdam
    from dogs_amd import densify
    from oracle import densify_oracle as D
    params, g = _params(N, 100 + N, hip_device)
    model = types.SimpleNamespace(percent_dense=0.01)
    for k, a in zip(densify.NAMES, densify.ATTRS):
        setattr(model, a, torch.nn.Parameter(params[k].clone()))
    opt = SparseGaussianAdam([{"params": [getattr(model, a)], "lr": LRS[k], "name": k}
                              for k, a in zip(densify.NAMES, densify.ATTRS)], lr=0.0, eps=1e-15)
    for a in densify.ATTRS:  # one step: non-trivial moments
        getattr(model, a).grad = torch.randn(getattr(model, a).shape, generator=g).to(hip_device)
    opt.step(torch.ones(N, dtype=torch.bool, device=hip_device), N)
    model.xyz_gradient_accum = (torch.rand((N, 1), generator=g) * 4e-4).to(hip_device)
    den = torch.randint(0, 3, (N, 1), generator=g).float()
    model.denom = den.to(hip_device)
    model.max_radii2D = (torch.rand(N, generator=g) * 40).to(hip_device)
    extent = 3.0
    before = {k: getattr(model, a).detach().cpu().numpy().copy() for k, a in zip(densify.NAMES, densify.ATTRS)}
    mom = {k: (opt.state[getattr(model, a)]["exp_avg"].cpu().numpy().copy(),
               opt.state[getattr(model, a)]["exp_avg_sq"].cpu().numpy().copy())
           for k, a in zip(densify.NAMES, densify.ATTRS)}
    stats_in = (model.xyz_gradient_accum.cpu().numpy().copy(), model.denom.cpu().numpy().copy(),
                model.max_radii2D.cpu().numpy().copy())
    drawn = []

    def normal(mean, std):
        s = torch.normal(mean=mean, std=std)
        drawn.append(s.cpu().numpy().copy())
        return s

    n_out = densify.densify_and_prune(model, 2e-4, 0.005, extent, screen, opt, bounding_box=bbox, normal=normal)
    samples = drawn[0] if drawn else np.zeros((0, 3), np.float32)
    out, mom_o, st_o = D.densify_and_prune(before, mom, *stats_in, 2e-4, 0.005, extent, screen, 0.01, samples,
                                           bounding_box=bbox)
    assert n_out == out["xyz"].shape[0]
    ns = samples.shape[0] // 2
    n_child = 2 * ns
    for k, a in zip(densify.NAMES, densify.ATTRS):
        p = getattr(model, a)
        assert isinstance(p, torch.nn.Parameter) and opt.param_groups[densify.NAMES.index(k)]["params"][0] is p
        h = p.detach().cpu().numpy()
        assert h.shape == out[k].shape, k
        if k in ("xyz", "scaling") and n_child:
            # rows of split children are the last n_child rows that survived the prune: compare with a tolerance
            np.testing.assert_allclose(h, out[k], rtol=2e-6, atol=1e-7, err_msg=k)
        else:
            np.testing.assert_array_equal(h, out[k], err_msg=k)
        st = opt.state[p]
        np.testing.assert_array_equal(st["exp_avg"].cpu().numpy(), mom_o[k][0], err_msg=k)
        np.testing.assert_array_equal(st["exp_avg_sq"].cpu().numpy(), mom_o[k][1], err_msg=k)
    for k, v in st_o.items():
        np.testing.assert_array_equal(getattr(model, k).cpu().numpy(), v, err_msg=k)
    if N > 1:
        assert ns > 0 and n_out != N  # the case exercised splitting and pruning
