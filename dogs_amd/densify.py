"""Densification on the GPU: the per-view statistics and densify_and_prune of
conerf/model/gaussian_fields/gaussian_splat_model.py, as drop-in functions over the reference's model object.

The model is duck-typed exactly as GaussianSplatModel stores it: `_xyz [N,3]`, `_features_dc [N,1,3]`,
`_features_rest [N,M,3]`, `_opacity [N,1]` (raw), `_scaling [N,3]` (raw), `_quaternion [N,4]` (raw),
`xyz_gradient_accum [N,1]`, `denom [N,1]`, `max_radii2D [N]`, `percent_dense`; the optimizer's groups are named
"xyz", "f_dc", "f_rest", "opacity", "scaling", "quaternion" (gaussian_splat_model.py:51-110).  A maintainer binds
them as methods:

    GaussianSplatModel.add_densification_stats = dogs_amd.densify.add_densification_stats
    GaussianSplatModel.densify_and_prune = dogs_amd.densify.densify_and_prune

The reference does densify_and_prune with ~40 boolean-mask indexing ops (each a device sync) and 3 rounds of
optimizer-state concatenation/masking; here it is one selection pass, one candidate pass and one gather
(dg_densify_* in include/dogs_hip.h), with two host syncs (the clone/split counts and the final count).
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.nn as nn

from . import _lib

NAMES = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "quaternion")
ATTRS = ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_quaternion")


def add_densification_stats(model, screen_space_points, update_filter, radii=None):
    """add_densification_stats (gaussian_splat_model.py:533-541); with `radii`, also the max_radii2D update the
    trainer does just before it (gaussian_trainer.py:433-436).  One launch (dg_add_densification_stats)."""
    grad = screen_space_points.grad if isinstance(screen_space_points, torch.Tensor) else screen_space_points
    N = int(model.xyz_gradient_accum.shape[0])
    vis = update_filter.contiguous()
    if vis.dtype != torch.bool:
        vis = vis.bool()
    dm = grad.reshape(N, -1).contiguous()
    if radii is None:  # statistics only: max_radii2D untouched (max with itself)
        mr = model.max_radii2D
        r = torch.zeros(N, dtype=torch.int32, device=vis.device)
    else:
        mr = model.max_radii2D
        r = radii.contiguous().int()
    for t, n in ((model.xyz_gradient_accum, "xyz_gradient_accum"), (model.denom, "denom"), (mr, "max_radii2D")):
        if not t.is_contiguous() or t.dtype != torch.float32:
            raise RuntimeError(f"{n} must be a contiguous float32 tensor (updated in place)")
    st = _lib.DgDensifyStats(r.data_ptr(), dm.data_ptr(), int(dm.stride(0)), mr.data_ptr(),
                             model.xyz_gradient_accum.data_ptr(), model.denom.data_ptr())
    with _lib.device_ctx(vis.device):
        _lib.check(_lib.load().dg_add_densification_stats(C.byref(st), vis.data_ptr(), N, _lib.stream_of(vis.device)))


def _group_of(optimizer, name):
    for g in optimizer.param_groups:
        if g.get("name") == name:
            return g
    return None


@torch.no_grad()
def densify_and_prune(model, max_grad, min_opacity, extent, max_screen_size, optimizer, bounding_box=None,
                      num_replica: int = 2, normal=torch.normal):
    """densify_and_prune (gaussian_splat_model.py:496-531) = densify_and_clone (:434-453) + densify_and_split
    (:455-494) + the opacity / bounding-box / size prune, with the reference's row order
    [originals not split | clones | split children (replica-major)] and its optimizer-state handling (appended rows
    get zero moments, cat_tensors_to_optimizer; pruned rows drop theirs, prune_optimizer).  `normal` draws the split
    offsets exactly as the reference (torch.normal(mean=0, std=stds)), so a seeded generator gives the same points.
    Afterwards the statistics are zeros, as densification_postfix leaves them (so, as in the reference, the
    max_radii2D > max_screen_size test never fires)."""
    params = [getattr(model, a) for a in ATTRS]
    dev = params[0].device
    N = int(params[0].shape[0])
    flat = [p.detach().reshape(N, -1).contiguous() if N else p.detach().reshape(0, 1) for p in params]
    widths = [int(f.shape[1]) if N else int(p[0].numel()) if p.shape[0] else 1 for f, p in zip(flat, params)]
    groups = [_group_of(optimizer, n) for n in NAMES]
    states = []
    for g in groups:
        st = optimizer.state.get(g["params"][0], None) if g is not None else None
        if st is not None and "exp_avg" in st:
            states.append((st["exp_avg"].reshape(N, -1).contiguous(), st["exp_avg_sq"].reshape(N, -1).contiguous()))
        else:
            states.append(None)
    ga = model.xyz_gradient_accum.reshape(-1).contiguous()
    dn = model.denom.reshape(-1).contiguous()

    a = _lib.DgDensifyArgs()
    a.set.N = N
    for q in range(6):
        a.set.params[q] = flat[q].data_ptr() if N else None
        a.set.exp_avg[q] = states[q][0].data_ptr() if (states[q] is not None and N) else None
        a.set.exp_avg_sq[q] = states[q][1].data_ptr() if (states[q] is not None and N) else None
        a.set.width[q] = widths[q]
    a.set.grad_accum, a.set.denom = (ga.data_ptr(), dn.data_ptr()) if N else (None, None)
    a.max_grad = float(max_grad)
    a.dense_extent = float(model.percent_dense * extent)
    a.replicas = int(num_replica)
    a.min_opacity = float(min_opacity)
    a.use_bbox = int(bounding_box is not None)
    a.bbox_z = float(bounding_box[2]) if bounding_box is not None else 0.0
    a.use_screen = int(max_screen_size is not None)
    a.max_screen_size = float(max_screen_size) if max_screen_size is not None else 0.0
    a.big_extent = float(0.1 * extent)

    L = _lib.load()
    arena = _lib.TensorArena(dev)
    s = _lib.stream_of(dev)
    with _lib.device_ctx(dev):
        _lib.check(L.dg_densify_select(C.byref(a), arena.fn, None, s))
        ns = int(a.ns)
        samples = None
        if ns:
            stds = torch.empty((num_replica * ns, 3), dtype=torch.float32, device=dev)
            _lib.check(L.dg_densify_split_stds(C.byref(a), stds.data_ptr(), s))
            means = torch.zeros((stds.size(0), 3), device=dev)
            samples = normal(mean=means, std=stds).contiguous()
            a.samples = samples.data_ptr()
        _lib.check(L.dg_densify_count(C.byref(a), arena.fn, None, s))
        n_out = int(a.n_out)
        outs, out_m, out_v = [], [], []
        for q in range(6):
            shape = (n_out,) + tuple(params[q].shape[1:])
            outs.append(torch.empty(shape, dtype=torch.float32, device=dev))
            has = states[q] is not None
            out_m.append(torch.empty(shape, dtype=torch.float32, device=dev) if has else None)
            out_v.append(torch.empty(shape, dtype=torch.float32, device=dev) if has else None)
            a.out_params[q] = outs[q].data_ptr() if n_out else None
            a.out_exp_avg[q] = out_m[q].data_ptr() if (has and n_out) else None
            a.out_exp_avg_sq[q] = out_v[q].data_ptr() if (has and n_out) else None
        _lib.check(L.dg_densify_gather(C.byref(a), s))
    del samples, flat, states, arena

    for q, (name, attr) in enumerate(zip(NAMES, ATTRS)):
        g = groups[q]
        newp = nn.Parameter(outs[q].requires_grad_(True))
        if g is not None:
            old = g["params"][0]
            stored = optimizer.state.pop(old, None)
            g["params"][0] = newp
            if stored is not None and out_m[q] is not None:
                stored["exp_avg"] = out_m[q]
                stored["exp_avg_sq"] = out_v[q]
                optimizer.state[newp] = stored
        setattr(model, attr, newp)
    model.xyz_gradient_accum = torch.zeros((n_out, 1), device=dev)
    model.denom = torch.zeros((n_out, 1), device=dev)
    model.max_radii2D = torch.zeros((n_out,), device=dev)
    return n_out
