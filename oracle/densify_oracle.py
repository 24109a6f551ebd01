"""numpy restatement of the reference's densification -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/.  The product path (dogs_amd/densify.py -> dg_densify_*) must never import it.

Follows conerf/model/gaussian_fields/gaussian_splat_model.py op by op:
  add_densification_stats :533-541 (+ the max_radii2D update of conerf/trainers/gaussian_trainer.py:433-436),
  densify_and_clone :434-453, densify_and_split :455-494, densify_and_prune :496-531,
  densification_postfix :369-395 with cat_tensors_to_optimizer :51-83, prune_points :397-411 with
  prune_optimizer :86-110, quaternion_to_rotation_mat / normalize_quaternion (utils.py:20-67).
Parity unpinned: the reference holds no tests or fixtures for these functions and its module
cannot be imported here (plyfile is absent); the split offsets are an input (the caller draws them
with torch.normal exactly as the reference does).

State layout: params / moments are dicts name -> float32 array [N, ...]; moments[name] is None when the optimizer
holds no state for that tensor.
"""
from __future__ import annotations

import numpy as np

NAMES = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "quaternion")
f32 = np.float32


def densification_stats(max_radii2D, grad_accum, denom, radii, screen_grad, update_filter):
    """gaussian_trainer.py:433-436 then add_densification_stats (participated_pixels = 1), in place."""
    vis = np.asarray(update_filter, bool)
    max_radii2D[vis] = np.maximum(max_radii2D[vis], radii[vis].astype(f32))
    g = screen_grad[vis, :2].astype(f32)
    grad_accum[vis] += np.sqrt(g[:, 0] * g[:, 0] + g[:, 1] * g[:, 1]).reshape(-1, 1).astype(f32)
    denom[vis] += f32(1.0)


def _sigmoid(x):
    return (f32(1.0) / (f32(1.0) + np.exp(-x))).astype(f32)


def _rot(q):
    """normalize_quaternion + quaternion_to_rotation_mat (utils.py:20-67)."""
    n = np.sqrt(((q[:, 0] * q[:, 0] + q[:, 1] * q[:, 1]) + q[:, 2] * q[:, 2]) + q[:, 3] * q[:, 3])
    qn = q / n[:, None]
    r, x, y, z = qn[:, 0], qn[:, 1], qn[:, 2], qn[:, 3]
    one, two = f32(1.0), f32(2.0)
    R = np.zeros((q.shape[0], 3, 3), f32)
    R[:, 0, 0] = one - two * (y * y + z * z)
    R[:, 0, 1] = two * (x * y - r * z)
    R[:, 0, 2] = two * (x * z + r * y)
    R[:, 1, 0] = two * (x * y + r * z)
    R[:, 1, 1] = one - two * (x * x + z * z)
    R[:, 1, 2] = two * (y * z - r * x)
    R[:, 2, 0] = two * (x * z - r * y)
    R[:, 2, 1] = two * (y * z + r * x)
    R[:, 2, 2] = one - two * (x * x + y * y)
    return R


def _postfix(params, moments, new):
    """densification_postfix / cat_tensors_to_optimizer: append rows, zero moments for them."""
    for k in NAMES:
        params[k] = np.concatenate([params[k], new[k]], 0)
        if moments[k] is not None:
            m, v = moments[k]
            moments[k] = (np.concatenate([m, np.zeros_like(new[k])], 0), np.concatenate([v, np.zeros_like(new[k])], 0))


def _prune(params, moments, stats, mask):
    """prune_points / prune_optimizer: keep ~mask."""
    keep = ~mask
    for k in NAMES:
        params[k] = params[k][keep]
        if moments[k] is not None:
            moments[k] = (moments[k][0][keep], moments[k][1][keep])
    for k in stats:
        stats[k] = stats[k][keep]


def densify_and_prune(params, moments, grad_accum, denom, max_radii2D, max_grad, min_opacity, extent,
                      max_screen_size, percent_dense, samples, bounding_box=None, num_replica=2):
    """Returns (params, moments, stats) after densify_and_prune; `samples` [num_replica*ns, 3] are the split
    offsets torch.normal drew.  Inputs are not modified."""
    params = {k: np.array(v, f32) for k, v in params.items()}
    moments = {k: (None if moments.get(k) is None else (np.array(moments[k][0], f32), np.array(moments[k][1], f32)))
               for k in NAMES}
    with np.errstate(invalid="ignore", divide="ignore"):
        grads = (grad_accum / denom).astype(f32)
    grads[np.isnan(grads)] = 0.0
    stats = {"xyz_gradient_accum": grad_accum.copy(), "denom": denom.copy(), "max_radii2D": max_radii2D.copy()}

    def get_scaling():
        return np.exp(params["scaling"]).astype(f32)

    # densify_and_clone (:434-453)
    sel = np.abs(grads[:, 0]) >= f32(max_grad)   # torch.norm over the size-1 last dim
    sel &= get_scaling().max(1) <= f32(percent_dense * extent)
    _postfix(params, moments, {k: params[k][sel] for k in NAMES})
    n1 = params["xyz"].shape[0]
    stats = {"xyz_gradient_accum": np.zeros((n1, 1), f32), "denom": np.zeros((n1, 1), f32),
             "max_radii2D": np.zeros((n1,), f32)}

    # densify_and_split (:455-494)
    padded = np.zeros((n1,), f32)
    padded[:grads.shape[0]] = grads[:, 0]
    sel = padded >= f32(max_grad)
    sel &= get_scaling().max(1) > f32(percent_dense * extent)
    ns = int(sel.sum())
    assert samples.shape == (num_replica * ns, 3), (samples.shape, ns)
    R = np.tile(_rot(params["quaternion"][sel]), (num_replica, 1, 1))
    s = samples.astype(f32)
    # bmm(R, s): a k = 3 fused multiply-add chain per entry (float64 products of float32 values rounded once
    # per step reproduce fmaf)
    dot = np.zeros((R.shape[0], 3), f32)
    for c in range(3):
        acc = (R[:, c, 0] * s[:, 0]).astype(f32)
        acc = (R[:, c, 1].astype(np.float64) * s[:, 1] + acc).astype(f32)
        acc = (R[:, c, 2].astype(np.float64) * s[:, 2] + acc).astype(f32)
        dot[:, c] = acc
    new_xyz = (dot + np.tile(params["xyz"][sel], (num_replica, 1))).astype(f32)
    inv = f32(1.0) / f32(0.8 * num_replica)   # torch on the GPU: division by a Python scalar = multiply by 1/x
    new_scaling = np.log((np.tile(get_scaling()[sel], (num_replica, 1)) * inv).astype(f32)).astype(f32)
    new = {"xyz": new_xyz, "scaling": new_scaling}
    for k in ("f_dc", "f_rest", "opacity", "quaternion"):
        new[k] = np.tile(params[k][sel], (num_replica,) + (1,) * (params[k].ndim - 1))
    _postfix(params, moments, new)
    n2 = params["xyz"].shape[0]
    stats = {"xyz_gradient_accum": np.zeros((n2, 1), f32), "denom": np.zeros((n2, 1), f32),
             "max_radii2D": np.zeros((n2,), f32)}
    _prune(params, moments, stats, np.concatenate([sel, np.zeros(num_replica * ns, bool)]))

    # prune (:516-528)
    prune = _sigmoid(params["opacity"]).reshape(-1) < f32(min_opacity)
    if bounding_box is not None:
        prune |= params["xyz"][:, 2] < f32(bounding_box[2])
    if max_screen_size is not None:
        big_vs = stats["max_radii2D"] > max_screen_size
        big_ws = get_scaling().max(1) > f32(0.1 * extent)
        prune = prune | big_vs | big_ws
    _prune(params, moments, stats, prune)
    return params, moments, stats
