"""GaussianSplatModel (conerf/model/gaussian_fields/gaussian_splat_model.py:120-726): the parameter set the training
loop mutates, with the reference's attribute names, getters and in-place lifecycle operations.

The tensors live on the device as the reference stores them (`_xyz [N,3]`, `_features_dc [N,1,3]`,
`_features_rest [N,M,3]`, `_scaling [N,3]` raw log, `_quaternion [N,4]` raw, `_opacity [N,1]` raw logit, plus
`xyz_gradient_accum [N,1]`, `denom [N,1]`, `max_radii2D [N]`).  The operations that replace them go through the
library instead of torch's boolean-mask indexing:

* densify_and_prune  -> dogs_amd.densify (dg_densify_*: one selection, one candidate pass, one gather);
* prune_points       -> dg_prune_select + dg_densify_gather + dg_prune_gather_stats (gaussian_splat_model.py:396-410:
                        every tensor, its Adam moments and the statistics compacted in one pass, one host sync);
* reset_opacity      -> :362-367, a new opacity tensor with fresh (zero) Adam moments (replace_tensor_to_optimizer).

After any of them the optimizer's groups hold new tensors: a dogs_amd.train_step.NativeTrainStep bound to the old
ones refuses to step until rebind() (its pointer check)."""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from .densify import ATTRS, NAMES

SH_C0 = 0.28209479177387814


def inverse_sigmoid(x: torch.Tensor) -> torch.Tensor:
    """gaussian_splat_model.py:27-31."""
    return torch.log(x / (1 - x))


def RGB2SH(rgb):  # noqa: N802  (sh_utils.py:115)
    return (rgb - 0.5) / SH_C0


class GaussianSplatModel:
    def __init__(self, max_sh_degree: int = 3, percent_dense: float = 0.01, device="cuda"):
        self.device = torch.device(device)
        self.active_sh_degree = 0
        self.max_sh_degree = max_sh_degree
        self.percent_dense = percent_dense
        e = torch.empty(0)
        self._xyz = self._features_dc = self._features_rest = e
        self._scaling = self._quaternion = self._opacity = e
        self.max_radii2D = self.xyz_gradient_accum = self.denom = e
        self._exposure = e
        self.image_id_to_index: dict = {}

    # ---- getters (gaussian_splat_model.py:156-259)
    @property
    def get_xyz(self):
        return self._xyz

    @property
    def get_features_dc(self):
        return self._features_dc

    @property
    def get_features_rest(self):
        return self._features_rest

    @property
    def get_features(self):
        return torch.cat((self._features_dc, self._features_rest), dim=1)

    @property
    def get_raw_scaling(self):
        return self._scaling

    @property
    def get_scaling(self):
        return torch.exp(self._scaling)

    @property
    def get_raw_quaternion(self):
        return self._quaternion

    @property
    def get_quaternion(self):
        return torch.nn.functional.normalize(self._quaternion)

    @property
    def get_raw_opacity(self):
        return self._opacity

    @property
    def get_opacity(self):
        return torch.sigmoid(self._opacity)

    @property
    def get_exposure(self):
        return self._exposure

    def get_exposure_from_id(self, image_id: int):
        """:272-273: the [3,4] affine colour transform of a training image."""
        return self._exposure[self.image_id_to_index[image_id]]

    def init_exposure(self, image_idxs) -> None:
        """init_from_colmap_pcd's trained-exposure part (:578-582): one identity [3,4] per training image index."""
        idxs = [int(i) for i in image_idxs]
        self.image_id_to_index = {idx: ind for ind, idx in enumerate(idxs)}
        exposure = torch.eye(3, 4, device=self.device)[None].repeat(len(idxs), 1, 1)
        self._exposure = nn.Parameter(exposure.requires_grad_(True))

    @property
    def num_gaussians(self) -> int:
        return int(self._xyz.shape[0])

    def params(self) -> dict:
        """{optimizer group name: tensor} in setup_optimizer's order (gaussian_trainer.py:205-230)."""
        return {n: getattr(self, a) for n, a in zip(NAMES, ATTRS)}

    def get_all_properties(self, indices: torch.Tensor | None = None) -> tuple:
        """:275-288 (xyz, f_dc, f_rest, scaling, quaternion, opacity)."""
        t = (self._xyz, self._features_dc, self._features_rest, self._scaling, self._quaternion, self._opacity)
        return t if indices is None else tuple(x[indices] for x in t)

    # ---- construction (:543-614)
    def _reset_stats(self):
        n = self.num_gaussians
        self.max_radii2D = torch.zeros((n,), device=self.device)
        self.xyz_gradient_accum = torch.zeros((n, 1), device=self.device)
        self.denom = torch.zeros((n, 1), device=self.device)

    def init_from_colmap_pcd(self, points, colors, image_idxs=None) -> None:
        """:543-587: SH dc from the point colours, rest zero, scales from simple-knn's mean squared 3-NN distance
        (distCUDA2 on the device), identity rotations, opacity 0.1; with image_idxs (appearance.use_trained_exposure)
        an identity exposure per training image."""
        from .simple_knn._C import distCUDA2
        pts = torch.as_tensor(np.asarray(points)).float().to(self.device)
        col = RGB2SH(torch.as_tensor(np.asarray(colors)).float().to(self.device))
        n = pts.shape[0]
        feats = torch.zeros((n, 3, (self.max_sh_degree + 1) ** 2), device=self.device)
        feats[:, :3, 0] = col
        dist2 = torch.clamp_min(distCUDA2(pts.contiguous()), 0.0000001)
        scales = torch.log(torch.sqrt(dist2))[..., None].repeat(1, 3)
        quats = torch.zeros((n, 4), device=self.device)
        quats[:, 0] = 1.0
        opac = inverse_sigmoid(0.1 * torch.ones((n, 1), dtype=torch.float, device=self.device))
        self._xyz = nn.Parameter(pts.requires_grad_(True))
        self._features_dc = nn.Parameter(feats[:, :, 0:1].transpose(1, 2).contiguous().requires_grad_(True))
        self._features_rest = nn.Parameter(feats[:, :, 1:].transpose(1, 2).contiguous().requires_grad_(True))
        self._scaling = nn.Parameter(scales.contiguous().requires_grad_(True))
        self._quaternion = nn.Parameter(quats.requires_grad_(True))
        self._opacity = nn.Parameter(opac.contiguous().requires_grad_(True))
        self._reset_stats()
        if image_idxs is not None:
            self.init_exposure(image_idxs)

    def init_from_external_properties(self, xyz, features_dc, features_rest, scaling, quaternion, opacity,
                                      optimizable: bool = False) -> None:
        """:589-614."""
        ts = (xyz, features_dc, features_rest, scaling, quaternion, opacity)
        ts = tuple(t.detach().to(self.device).contiguous() for t in ts)
        if optimizable:
            ts = tuple(nn.Parameter(t.requires_grad_(True)) for t in ts)
        (self._xyz, self._features_dc, self._features_rest, self._scaling, self._quaternion,
         self._opacity) = ts
        self._reset_stats()

    def get_sub_gaussians(self, indices: torch.Tensor) -> "GaussianSplatModel":
        """:290-306: a new optimisable model of the given rows with zero statistics."""
        sub = GaussianSplatModel(self.max_sh_degree, self.percent_dense, self.device)
        sub.active_sh_degree = self.active_sh_degree
        idx = indices.to(self.device)
        sub.init_from_external_properties(*(t[idx] for t in self.get_all_properties()), optimizable=True)
        return sub

    def extract_sub_gaussians(self, indices=None) -> None:
        """:308-314 (the statistics are left as they are, as in the reference)."""
        idx = indices.to(self.device) if isinstance(indices, torch.Tensor) else indices
        for a in ATTRS:
            setattr(self, a, getattr(self, a)[idx])

    def increase_SH_degree(self) -> None:  # noqa: N802  (:358-360)
        if self.active_sh_degree < self.max_sh_degree:
            self.active_sh_degree += 1

    # ---- lifecycle operations that replace the optimised tensors
    @torch.no_grad()
    def reset_opacity(self, optimizer) -> None:
        """:362-367: opacity = inverse_sigmoid(min(sigmoid(opacity), 0.01)), with zero Adam moments
        (replace_tensor_to_optimizer, :34-48)."""
        new = inverse_sigmoid(torch.min(self.get_opacity, torch.ones_like(self.get_opacity) * 0.01))
        for g in optimizer.param_groups:
            if g["name"] != "opacity":
                continue
            st = optimizer.state.get(g["params"][0], None)
            if st is None:
                st = {"step": torch.tensor(0.0, dtype=torch.float32)}
            st["exp_avg"] = torch.zeros_like(new)
            st["exp_avg_sq"] = torch.zeros_like(new)
            optimizer.state.pop(g["params"][0], None)
            g["params"][0] = nn.Parameter(new.contiguous().requires_grad_(True))
            optimizer.state[g["params"][0]] = st
            self._opacity = g["params"][0]

    def densify_and_prune(self, max_grad, min_opacity, extent, max_screen_size, optimizer, bounding_box=None):
        """:501-531 on the device (dogs_amd.densify)."""
        from .densify import densify_and_prune
        return densify_and_prune(self, max_grad, min_opacity, extent, max_screen_size, optimizer, bounding_box)

    def add_densification_stats(self, screen_space_points, update_filter, radii=None):
        """:533-541 (+ the trainer's max_radii2D update when radii is given), one launch."""
        from .densify import add_densification_stats
        add_densification_stats(self, screen_space_points, update_filter, radii)

    @torch.no_grad()
    def prune_points(self, mask: torch.Tensor, optimizer=None) -> int:
        """:396-410 (with prune_optimizer :86-108): drop the rows where mask is True from every tensor, its Adam
        moments and the statistics.  optimizer None: the tensors only (prune_gaussians, :420-432).  One host sync."""
        return _compact(self, mask, optimizer)

    @torch.no_grad()
    def prune_gaussians_with_opt(self, percent: float, import_score: torch.Tensor, optimizer) -> int:
        """:412-418: prune every Gaussian whose score is <= the score at index int(percent (N - 1)) of the sorted
        scores."""
        return self.prune_points(percentile_mask(import_score, percent), optimizer)

    @torch.no_grad()
    def prune_gaussians(self, percent: float, import_score: torch.Tensor) -> int:
        """:420-432: the same selection on a non-optimised model (no optimizer state)."""
        return self.prune_points(percentile_mask(import_score, percent), None)


def percentile_mask(import_score: torch.Tensor, percent: float) -> torch.Tensor:
    """prune_gaussians_with_opt's selection (gaussian_splat_model.py:413-416), on the device, no host sync."""
    sorted_tensor, _ = torch.sort(import_score, dim=0)
    idx = int(percent * (sorted_tensor.shape[0] - 1))
    return (import_score <= sorted_tensor[idx]).squeeze()


def _compact(model, mask: torch.Tensor, optimizer) -> int:
    params = [getattr(model, a) for a in ATTRS]
    dev = params[0].device
    N = int(params[0].shape[0])
    if N == 0:
        return 0
    mask = mask.reshape(-1)
    if mask.numel() != N:
        raise RuntimeError(f"prune mask has {mask.numel()} entries for {N} Gaussians")
    pm = mask.to(device=dev, dtype=torch.uint8).contiguous()
    flat = [p.detach().reshape(N, -1).contiguous() for p in params]
    groups = {g.get("name"): g for g in optimizer.param_groups} if optimizer is not None else {}
    states = []
    for n in NAMES:
        g = groups.get(n)
        st = optimizer.state.get(g["params"][0], None) if g is not None else None
        if st is not None and "exp_avg" in st:
            states.append((st["exp_avg"].reshape(N, -1).contiguous(), st["exp_avg_sq"].reshape(N, -1).contiguous()))
        else:
            states.append(None)
    have_stats = (isinstance(model.xyz_gradient_accum, torch.Tensor) and model.xyz_gradient_accum.numel() == N
                  and model.denom.numel() == N and model.max_radii2D.numel() == N)
    ga = model.xyz_gradient_accum.reshape(-1).contiguous() if have_stats else None
    dn = model.denom.reshape(-1).contiguous() if have_stats else None
    mr = model.max_radii2D.reshape(-1).float().contiguous() if have_stats else None

    a = _lib.DgDensifyArgs()
    a.set.N = N
    for q in range(6):
        a.set.params[q] = flat[q].data_ptr()
        a.set.exp_avg[q] = states[q][0].data_ptr() if states[q] is not None else None
        a.set.exp_avg_sq[q] = states[q][1].data_ptr() if states[q] is not None else None
        a.set.width[q] = int(flat[q].shape[1])
    a.set.grad_accum, a.set.denom = (ga.data_ptr(), dn.data_ptr()) if have_stats else (None, None)
    L = _lib.load()
    arena = _lib.TensorArena(dev)
    s = _lib.stream_of(dev)
    with _lib.device_ctx(dev):
        _lib.check(L.dg_prune_select(C.byref(a), pm.data_ptr(), arena.fn, None, s))
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
        if have_stats:
            oga = torch.empty((n_out, 1), device=dev)
            odn = torch.empty((n_out, 1), device=dev)
            omr = torch.empty((n_out,), device=dev)
            _lib.check(L.dg_prune_gather_stats(C.byref(a), mr.data_ptr(), oga.data_ptr(), odn.data_ptr(),
                                               omr.data_ptr(), s))
    del flat, arena
    for q, (name, attr) in enumerate(zip(NAMES, ATTRS)):
        old = getattr(model, attr)
        newp = nn.Parameter(outs[q].requires_grad_(True)) if isinstance(old, nn.Parameter) or optimizer is not None \
            else outs[q]
        g = groups.get(name)
        if g is not None:
            stored = optimizer.state.pop(g["params"][0], None)
            g["params"][0] = newp
            if stored is not None and out_m[q] is not None:
                stored["exp_avg"], stored["exp_avg_sq"] = out_m[q], out_v[q]
                optimizer.state[newp] = stored
        setattr(model, attr, newp)
    if have_stats:
        model.xyz_gradient_accum, model.denom, model.max_radii2D = oga, odn, omr
    return n_out
