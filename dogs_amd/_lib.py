"""ctypes binding of libdogs_hip.so (include/dogs_hip.h).

This is the only way the Python layer reaches the GPU kernels.  There is no CPU fallback: if the
library is missing or a tensor is not on a HIP device, calls raise.
"""
from __future__ import annotations

import contextlib
import atexit
import ctypes as C
import os
import threading
import weakref

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_lib", "libdogs_hip.so")

_f32p = C.POINTER(C.c_float)


class DgRasterArgs(C.Structure):
    _fields_ = [
        ("P", C.c_int), ("D", C.c_int), ("M", C.c_int), ("W", C.c_int), ("H", C.c_int),
        ("prefiltered", C.c_int), ("antialiasing", C.c_int), ("debug", C.c_int), ("prefix_per_tile", C.c_int),
        ("scale_modifier", C.c_float), ("tanfovx", C.c_float), ("tanfovy", C.c_float),
        ("bg", C.c_void_p), ("means3D", C.c_void_p), ("colors", C.c_void_p), ("opacities", C.c_void_p),
        ("scales", C.c_void_p), ("rotations", C.c_void_p), ("cov3D_precomp", C.c_void_p),
        ("viewmatrix", C.c_void_p), ("projmatrix", C.c_void_p), ("dc", C.c_void_p), ("sh", C.c_void_p),
        ("campos", C.c_void_p), ("capacity_ctx", C.c_int),
    ]


class DgAdamGroup(C.Structure):
    _fields_ = [("param", C.c_void_p), ("grad", C.c_void_p), ("exp_avg", C.c_void_p), ("exp_avg_sq", C.c_void_p),
                ("lr", C.c_float), ("eps", C.c_float), ("M", C.c_uint32)]


class DgAdamProx(C.Structure):
    _fields_ = [("u", C.c_void_p), ("z", C.c_void_p), ("coef", C.c_float)]


class DgDensifyStats(C.Structure):
    _fields_ = [("radii", C.c_void_p), ("dmeans2D", C.c_void_p), ("dmeans2D_stride", C.c_uint32),
                ("max_radii2D", C.c_void_p), ("grad_accum", C.c_void_p), ("denom", C.c_void_p)]


class DgTrainStepArgs(C.Structure):
    _fields_ = [("view", DgRasterArgs), ("gt", C.c_void_p), ("lambda_dssim", C.c_float), ("lambda_scale", C.c_float),
                ("groups", DgAdamGroup * 6), ("prox", DgAdamProx * 6), ("stats", C.c_void_p), ("radii", C.c_void_p),
                ("image", C.c_void_p), ("loss", C.c_void_p), ("sh_status", C.c_void_p), ("mask", C.c_void_p),
                ("dmask", C.c_void_p), ("lambda_mask", C.c_float), ("depth_threshold", C.c_float)]


class DgGaussianSet(C.Structure):
    _fields_ = [("N", C.c_uint32), ("params", C.c_void_p * 6), ("exp_avg", C.c_void_p * 6),
                ("exp_avg_sq", C.c_void_p * 6), ("width", C.c_uint32 * 6), ("grad_accum", C.c_void_p),
                ("denom", C.c_void_p)]


class DgDensifyArgs(C.Structure):
    _fields_ = [("set", DgGaussianSet), ("max_grad", C.c_float), ("dense_extent", C.c_float),
                ("replicas", C.c_uint32), ("min_opacity", C.c_float), ("use_bbox", C.c_int), ("bbox_z", C.c_float),
                ("use_screen", C.c_int), ("max_screen_size", C.c_float), ("big_extent", C.c_float),
                ("samples", C.c_void_p), ("out_params", C.c_void_p * 6), ("out_exp_avg", C.c_void_p * 6),
                ("out_exp_avg_sq", C.c_void_p * 6), ("state", C.c_void_p), ("state2", C.c_void_p),
                ("nc", C.c_uint32), ("ns", C.c_uint32), ("n_out", C.c_uint32)]


ALLOC_FN = C.CFUNCTYPE(C.c_void_p, C.c_void_p, C.c_int, C.c_uint64)
DG_BUF_GEOM, DG_BUF_BINNING, DG_BUF_IMAGE, DG_BUF_BACKWARD, DG_BUF_TEMP, DG_BUF_BINNING2, DG_BUF_DENSIFY, \
    DG_BUF_DENSIFY2 = range(8)
DG_BUF_MEMBERS = 8


class DgFixedBuffer(C.Structure):
    """dg_fixed_buffer: the user argument of dg_fixed_alloc."""
    _fields_ = [("ptr", C.c_void_p), ("bytes", C.c_uint64)]


_FIXED_FN = None


def fixed_alloc_fn():
    """dg_fixed_alloc as a dg_alloc_fn argument: a C function pointer, so the library's allocation request does not
    call back into Python."""
    global _FIXED_FN
    if _FIXED_FN is None:
        _FIXED_FN = ALLOC_FN(C.cast(load().dg_fixed_alloc, C.c_void_p).value)
    return _FIXED_FN
DG_MAX_BOXES = 64


class DgBox2dSet(C.Structure):
    _fields_ = [("C", C.c_uint32), ("has_T", C.c_int), ("T", C.c_double * 6),
                ("box", (C.c_double * 4) * DG_MAX_BOXES)]

EXPORTS = ("dg_rasterize_forward", "dg_rasterize_backward", "dg_rasterize_count", "dg_mark_visible", "dg_rasterize_filter",
           "dg_cull_log_threshold", "dg_adaptive_capacity_ctx", "dg_release_capacity_context", "dg_capacity_contexts", "dg_conv3x3_wgrad", "dg_conv3x3_wgrad_scratch_bytes",
           "dg_conv3x3",
           "dg_mask_head_forward", "dg_mask_head_backward", "dg_mask_head_scratch_bytes", "dg_mask_head_nparams",
           "dg_adam_update", "dg_fused_ssim_forward", "dg_fused_ssim_backward", "dg_fused_ssim_parts",
           "dg_fused_ssim_mean", "dg_fused_ssim_mean_backward", "dg_mean_of_parts", "dg_dist_cuda2",
           "dg_geom_bytes", "dg_image_bytes", "dg_binning_bytes", "dg_backward_scratch_bytes", "dg_fixed_alloc",
           "dg_debug_sorted_instances",
           "dg_debug_geometry", "dg_debug_image_state", "dg_sort_pairs_u32", "dg_exclusive_scan_u32",
           "dg_profile_enable", "dg_profile_collect", "dg_binned_instances", "dg_adam_update_groups",
           "dg_add_densification_stats", "dg_densify_select", "dg_densify_split_stds", "dg_densify_count",
           "dg_densify_gather", "dg_splat_pack", "dg_ply_pack", "dg_ring_create", "dg_ring_submit", "dg_ring_next",
           "dg_ring_upload", "dg_ring_pending", "dg_ring_destroy", "dg_image_u8_to_chw", "dg_points_in_boxes2d", "dg_activate_forward", "dg_activate_backward", "dg_clamp_l1_blocks",
           "dg_clamp_l1_forward", "dg_clamp_l1_backward", "dg_row_prod_forward", "dg_row_prod_backward", "dg_adaptive_capacity", "dg_debug_counters", "dg_adam_update_groups_prox", "dg_train_step", "dg_train_sync",
           "dg_colmap_cameras", "dg_colmap_images", "dg_colmap_points3d", "dg_prune_select", "dg_prune_gather_stats",
           "dg_last_error", "dg_version", "dg_host_wait_ns", "dg_shutdown")

_lib = None
_lock = threading.Lock()


def load(path: str | None = None):
    """Load (once) and type the library.  Raises ImportError when it is not built."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or os.environ.get("DOGS_HIP_LIB") or LIB_PATH  # env override: A/B of two builds on one box
        if not os.path.exists(p):
            raise ImportError(f"libdogs_hip.so not found at {p}: build it with "
                              "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
        L = C.CDLL(p)
        vp, i64p = C.c_void_p, C.POINTER(C.c_int64)
        L.dg_rasterize_forward.restype = C.c_int
        L.dg_rasterize_forward.argtypes = [C.POINTER(DgRasterArgs), vp, vp, vp, ALLOC_FN, vp,
                                           C.POINTER(vp), C.POINTER(vp), C.POINTER(vp), C.POINTER(vp), i64p, i64p,
                                           vp]
        if hasattr(L, "dg_rasterize_count"):  # absent in older builds used for A/B runs
            L.dg_rasterize_count.restype = C.c_int
            L.dg_rasterize_count.argtypes = [C.POINTER(DgRasterArgs), vp, vp, vp, vp, ALLOC_FN, vp, i64p, vp]
        L.dg_rasterize_backward.restype = C.c_int
        L.dg_rasterize_backward.argtypes = [C.POINTER(DgRasterArgs), vp, vp, vp, vp, vp, C.c_int64, C.c_int64, vp, vp,
                                            vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, ALLOC_FN, vp, vp]
        L.dg_mark_visible.restype = C.c_int
        L.dg_mark_visible.argtypes = [C.c_int, vp, vp, vp, vp, vp]
        L.dg_rasterize_filter.restype = C.c_int
        L.dg_cull_log_threshold.restype = C.c_int
        L.dg_conv3x3_wgrad_scratch_bytes.restype = C.c_size_t
        L.dg_conv3x3_wgrad_scratch_bytes.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int]
        L.dg_conv3x3_wgrad.restype = C.c_int
        L.dg_mask_head_forward.restype = C.c_int
        L.dg_mask_head_forward.argtypes = [C.c_int] * 4 + [vp] * 7 + [vp]
        L.dg_mask_head_backward.restype = C.c_int
        L.dg_mask_head_backward.argtypes = [C.c_int] * 4 + [vp] * 10 + [C.c_size_t, vp]
        L.dg_mask_head_scratch_bytes.restype = C.c_size_t
        L.dg_mask_head_scratch_bytes.argtypes = [C.c_int, C.c_int]
        L.dg_mask_head_nparams.restype = C.c_int
        L.dg_conv3x3_wgrad.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, vp, vp, vp, C.c_int, vp, vp, vp,
                                       C.c_size_t, vp]
        L.dg_conv3x3.restype = C.c_int
        L.dg_conv3x3.argtypes = [C.c_int] * 4 + [vp] * 4 + [C.c_int, vp, vp]
        L.dg_cull_log_threshold.argtypes = [C.c_int64, vp, vp, vp]
        L.dg_rasterize_filter.argtypes = [C.POINTER(DgRasterArgs), vp, vp]
        L.dg_adam_update.restype = C.c_int
        L.dg_adam_update.argtypes = [vp, vp, vp, vp, vp, C.c_float, C.c_float, C.c_float, C.c_float,
                                     C.c_uint32, C.c_uint32, vp]
        L.dg_fused_ssim_forward.restype = C.c_int
        L.dg_fused_ssim_forward.argtypes = [C.c_int] * 4 + [C.c_float, C.c_float] + [vp] * 6 + [vp]
        L.dg_fused_ssim_backward.restype = C.c_int
        L.dg_fused_ssim_backward.argtypes = [C.c_int] * 4 + [C.c_float, C.c_float] + [vp] * 7 + [vp]
        L.dg_fused_ssim_parts.restype = C.c_uint32
        L.dg_fused_ssim_parts.argtypes = [C.c_int] * 4
        L.dg_fused_ssim_mean.restype = C.c_int
        L.dg_fused_ssim_mean.argtypes = [C.c_int] * 4 + [C.c_float, C.c_float] + [vp] * 7 + [vp]
        L.dg_fused_ssim_mean_backward.restype = C.c_int
        L.dg_fused_ssim_mean_backward.argtypes = [C.c_int] * 4 + [vp] * 7 + [vp]
        L.dg_mean_of_parts.restype = C.c_int
        L.dg_mean_of_parts.argtypes = [vp, C.c_uint32, C.c_uint32, vp, vp]
        L.dg_dist_cuda2.restype = C.c_int
        L.dg_dist_cuda2.argtypes = [C.c_int, vp, vp, ALLOC_FN, vp, vp]
        L.dg_geom_bytes.restype = C.c_uint64
        L.dg_geom_bytes.argtypes = [C.c_int]
        L.dg_image_bytes.restype = C.c_uint64
        L.dg_image_bytes.argtypes = [C.c_int, C.c_int]
        L.dg_binning_bytes.restype = C.c_uint64
        L.dg_binning_bytes.argtypes = [C.c_int64, C.c_int, C.c_int]
        L.dg_backward_scratch_bytes.restype = C.c_uint64
        L.dg_backward_scratch_bytes.argtypes = [C.POINTER(DgRasterArgs), C.c_int64]
        L.dg_debug_sorted_instances.restype = C.c_int
        L.dg_debug_sorted_instances.argtypes = [C.POINTER(DgRasterArgs), vp, vp, vp, vp, C.c_int64, C.c_int64,
                                                vp, vp, i64p, vp]
        if hasattr(L, "dg_binned_instances"):  # introspection only; absent in older builds used for A/B runs
            L.dg_binned_instances.restype = C.c_int
            L.dg_binned_instances.argtypes = [vp, C.c_int, i64p, vp]
        if hasattr(L, "dg_colmap_points3d"):
            u64p = C.POINTER(C.c_uint64)
            L.dg_colmap_cameras.restype = C.c_int
            L.dg_colmap_cameras.argtypes = [C.c_char_p, u64p, vp, vp, vp, vp]
            L.dg_colmap_images.restype = C.c_int
            L.dg_colmap_images.argtypes = [C.c_char_p, u64p, u64p, u64p, vp, vp, vp, vp, vp, vp, vp, vp]
            L.dg_colmap_points3d.restype = C.c_int
            L.dg_colmap_points3d.argtypes = [C.c_char_p, C.c_int, u64p, u64p, vp, vp, vp, vp, vp, vp]
        if hasattr(L, "dg_train_step"):
            L.dg_train_step.restype = C.c_int
            L.dg_train_step.argtypes = [C.POINTER(DgTrainStepArgs), ALLOC_FN, vp, vp]
        if hasattr(L, "dg_train_sync"):
            L.dg_train_sync.restype = C.c_int
            L.dg_train_sync.argtypes = [vp]
        if hasattr(L, "dg_debug_counters"):
            L.dg_debug_counters.restype = C.c_int
            L.dg_debug_counters.argtypes = [vp, C.c_int, C.POINTER(C.c_uint32), vp]
        if hasattr(L, "dg_adaptive_capacity"):
            L.dg_adaptive_capacity.restype = C.c_int
            L.dg_adaptive_capacity.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int)]
            L.dg_adaptive_capacity_ctx.restype = C.c_int
            L.dg_adaptive_capacity_ctx.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int)]
            L.dg_release_capacity_context.restype = C.c_int
            L.dg_release_capacity_context.argtypes = [C.c_int]
            L.dg_capacity_contexts.restype = C.c_int
            L.dg_capacity_contexts.argtypes = [C.POINTER(C.c_int)]
        L.dg_debug_geometry.restype = C.c_int
        L.dg_debug_geometry.argtypes = [vp, C.c_int, vp, vp, vp, vp, vp]
        L.dg_debug_image_state.restype = C.c_int
        L.dg_debug_image_state.argtypes = [vp, C.c_int, C.c_int, vp, vp, vp, vp, vp]
        L.dg_sort_pairs_u32.restype = C.c_int
        L.dg_sort_pairs_u32.argtypes = [vp, vp, C.c_uint32, C.c_int, C.c_int, ALLOC_FN, vp, vp]
        L.dg_exclusive_scan_u32.restype = C.c_int
        L.dg_exclusive_scan_u32.argtypes = [vp, vp, C.c_uint32, vp, ALLOC_FN, vp, vp]
        L.dg_profile_enable.restype = None
        L.dg_profile_enable.argtypes = [C.c_int]
        L.dg_profile_collect.restype = C.c_int
        L.dg_profile_collect.argtypes = [C.c_char_p, C.c_int]
        if hasattr(L, "dg_adam_update_groups"):  # absent in older builds used for A/B runs
            L.dg_adam_update_groups.restype = C.c_int
            L.dg_adam_update_groups.argtypes = [C.POINTER(DgAdamGroup), C.c_int, vp, C.c_uint32, C.c_float,
                                                C.c_float, C.POINTER(DgDensifyStats), vp]
            if hasattr(L, "dg_adam_update_groups_prox"):
                L.dg_adam_update_groups_prox.restype = C.c_int
                L.dg_adam_update_groups_prox.argtypes = [C.POINTER(DgAdamGroup), C.POINTER(DgAdamProx), C.c_int, vp,
                                                         C.c_uint32, C.c_float, C.c_float, C.POINTER(DgDensifyStats),
                                                         vp]
            L.dg_add_densification_stats.restype = C.c_int
            L.dg_add_densification_stats.argtypes = [C.POINTER(DgDensifyStats), vp, C.c_uint32, vp]
            dp = C.POINTER(DgDensifyArgs)
            L.dg_densify_select.restype = C.c_int
            L.dg_densify_select.argtypes = [dp, ALLOC_FN, vp, vp]
            L.dg_densify_split_stds.restype = C.c_int
            L.dg_densify_split_stds.argtypes = [dp, vp, vp]
            L.dg_densify_count.restype = C.c_int
            L.dg_densify_count.argtypes = [dp, ALLOC_FN, vp, vp]
            L.dg_densify_gather.restype = C.c_int
            L.dg_densify_gather.argtypes = [dp, vp]
            if hasattr(L, "dg_prune_select"):
                L.dg_prune_select.restype = C.c_int
                L.dg_prune_select.argtypes = [dp, vp, ALLOC_FN, vp, vp]
                L.dg_prune_gather_stats.restype = C.c_int
                L.dg_prune_gather_stats.argtypes = [dp, vp, vp, vp, vp, vp]
        if hasattr(L, "dg_splat_pack"):
            L.dg_splat_pack.restype = C.c_int
            L.dg_splat_pack.argtypes = [C.c_uint32, vp, vp, vp, vp, vp, vp, ALLOC_FN, vp, vp]
            L.dg_ply_pack.restype = C.c_int
            L.dg_ply_pack.argtypes = [C.c_uint32, vp, vp, vp, vp]
        if hasattr(L, "dg_clamp_l1_forward"):
            L.dg_clamp_l1_blocks.restype = C.c_uint32
            L.dg_clamp_l1_blocks.argtypes = [C.c_uint32]
            L.dg_clamp_l1_forward.restype = C.c_int
            L.dg_clamp_l1_forward.argtypes = [C.c_uint32] + [vp] * 4 + [vp]
            L.dg_clamp_l1_backward.restype = C.c_int
            L.dg_clamp_l1_backward.argtypes = [C.c_uint32] + [vp] * 6 + [vp]
            L.dg_row_prod_forward.restype = C.c_int
            L.dg_row_prod_forward.argtypes = [C.c_uint32, C.c_uint32, vp, vp, vp, C.c_uint32, vp]
            L.dg_row_prod_backward.restype = C.c_int
            L.dg_row_prod_backward.argtypes = [C.c_uint32, C.c_uint32] + [vp] * 4 + [C.c_uint32, vp, vp]
        if hasattr(L, "dg_activate_forward"):
            L.dg_activate_forward.restype = C.c_int
            L.dg_activate_forward.argtypes = [C.c_uint32] + [vp] * 6 + [vp]
            L.dg_activate_backward.restype = C.c_int
            L.dg_activate_backward.argtypes = [C.c_uint32] + [vp] * 9 + [vp]
        if hasattr(L, "dg_points_in_boxes2d"):
            L.dg_points_in_boxes2d.restype = C.c_int
            L.dg_points_in_boxes2d.argtypes = [C.c_uint32, vp, C.c_uint32, C.POINTER(DgBox2dSet), vp, vp,
                                               C.POINTER(C.c_uint32), C.c_int, ALLOC_FN, vp, vp]
        if hasattr(L, "dg_ring_create"):
            ip = C.POINTER(C.c_int)
            L.dg_ring_create.restype = vp
            L.dg_ring_create.argtypes = [C.c_int, C.c_uint64, C.c_int]
            L.dg_ring_submit.restype = C.c_int
            L.dg_ring_submit.argtypes = [vp, C.c_char_p, C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_int]
            L.dg_ring_next.restype = C.c_int
            L.dg_ring_next.argtypes = [vp, ip, ip, ip, ip, ip]
            L.dg_ring_upload.restype = C.c_int
            L.dg_ring_upload.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, vp, vp]
            L.dg_ring_pending.restype = C.c_int
            L.dg_ring_pending.argtypes = [vp]
            L.dg_ring_destroy.restype = None
            L.dg_ring_destroy.argtypes = [vp]
            L.dg_image_u8_to_chw.restype = C.c_int
            L.dg_image_u8_to_chw.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, vp, vp]
        L.dg_last_error.restype = C.c_char_p
        L.dg_last_error.argtypes = []
        L.dg_version.restype = C.c_int
        L.dg_host_wait_ns.restype = C.c_uint64
        L.dg_host_wait_ns.argtypes = []
        if hasattr(L, "dg_shutdown"):  # absent in older builds used for A/B runs
            L.dg_shutdown.restype = C.c_int
            L.dg_shutdown.argtypes = []
            # the library's side streams, probes, pinned counters and events go before the HIP runtime (and a
            # profiler's tool library) finalise: Python's atexit runs ahead of the C++ static destructors
            atexit.register(L.dg_shutdown)
        if path is None:
            _lib = L
        return L


def check(rc: int) -> None:
    if rc != 0:
        msg = load().dg_last_error()
        raise RuntimeError(msg.decode() if msg else "libdogs_hip call failed")


def ptr(t: torch.Tensor | None):
    """Device pointer of a tensor; None/empty -> NULL (the reference's 'empty tensor = absent')."""
    if t is None or t.numel() == 0:
        return None
    return t.data_ptr()


def require_device(t: torch.Tensor, name: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a HIP (cuda) tensor: libdogs_hip has no CPU path")


def require_f32_on(device: torch.device, **tensors: torch.Tensor) -> None:
    """Every tensor float32 and on `device` (a HIP device): the kernels read raw fp32 device pointers, so a host,
    foreign-device or other-dtype tensor would be read as garbage or fault instead of raising like torch's ops."""
    for name, t in tensors.items():
        require_device(t, name)
        if t.device != device:
            raise RuntimeError(f"{name} is on {t.device}, expected {device}")
        if t.dtype != torch.float32:
            raise RuntimeError(f"{name} must be float32, got {t.dtype}")


def stream_of(device: torch.device):
    """The raw HIP stream torch's current stream on `device` wraps (torch.cuda.current_stream(device).cuda_stream
    without building the Stream object: ~0.3 us instead of ~5 us, and a training step calls this about ten times)."""
    if _RAW_STREAM is None:  # a torch without the private accessor
        return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)
    idx = device.index if device.index is not None else torch._C._cuda_getDevice()
    return C.c_void_p(_RAW_STREAM(idx))


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


_SAME_DEVICE = contextlib.nullcontext()


def device_ctx(device: torch.device):
    """torch.cuda.device(device), or a no-op when it is already the current device (the usual case: entering and
    leaving the context costs a few us per call)."""
    if device.index is None or device.index == torch.cuda.current_device():
        return _SAME_DEVICE
    return torch.cuda.device(device)


def _bucket(n: int) -> int:
    """n rounded up to a multiple of 1/8 of its power of two (at most 12.5% more) above 1 MiB."""
    if n <= 1 << 20:
        return n
    q = 1 << (n.bit_length() - 4)
    return (n + q - 1) // q * q


# One ctypes callback for every arena: creating a CFUNCTYPE object per call was a measurable part of each forward /
# backward's host time.  An arena's `fn` makes it the calling thread's current arena and returns the shared callback;
# the library calls it synchronously, on the same thread, during the C call the pointer was passed to.
_TLS = threading.local()


def _arena_dispatch(user, which, nbytes):  # noqa: ARG001
    return _TLS.arena()._alloc(int(which), max(int(nbytes), 1))


_ARENA_FN = ALLOC_FN(_arena_dispatch)


class TensorArena:
    """dg_alloc_fn backed by the torch caching allocator; keeps the uint8 tensors per buffer kind."""

    def __init__(self, device: torch.device):
        self.device = device
        self.buffers: dict[int, torch.Tensor] = {}

    @property
    def fn(self):
        _TLS.arena = weakref.ref(self)   # weak: the thread does not keep the last call's buffers alive
        return _ARENA_FN

    def _alloc(self, which: int, n: int):
        try:
            # the per-view sizes (phase-2 binning, backward scratch: num_rendered) vary view to view and drift as a
            # scene trains; requests rounded up to an eighth of their power of two let the caching allocator hand
            # cached blocks back instead of a hipMalloc every few views (~40 us of host each)
            t = torch.empty(_bucket(n), dtype=torch.uint8, device=self.device)[:n]
        except Exception:  # noqa: BLE001 - reported to C as NULL, surfaces as RuntimeError
            return None
        self.buffers[which] = t
        return t.data_ptr()

    def get(self, which: int) -> torch.Tensor:
        return self.buffers.get(which, torch.empty(0, dtype=torch.uint8, device=self.device))


class ReuseArena:
    """dg_alloc_fn for a loop of same-shaped calls on one stream (the native training step): one grow-only uint8
    tensor per buffer kind, handed out again while it is large enough.  Stream order makes the reuse safe: the next
    call's kernels run after this call's on the same stream."""

    def __init__(self, device: torch.device, keep_retired: bool = False):
        self.device = device
        self.buffers: dict[int, torch.Tensor] = {}
        # keep_retired: outgrown buffers stay alive until release_retired() (work on a side stream may still read
        # them: the native step's overlapped update)
        self.keep_retired, self.retired = keep_retired, []

    @property
    def fn(self):
        _TLS.arena = weakref.ref(self)   # weak: the thread does not keep the last call's buffers alive
        return _ARENA_FN

    def _alloc(self, which: int, nbytes: int):
        t = self.buffers.get(which)
        if t is None or t.numel() < nbytes:
            try:
                nt = torch.empty(nbytes + nbytes // 4, dtype=torch.uint8, device=self.device)
            except Exception:  # noqa: BLE001 - reported to C as NULL, surfaces as RuntimeError
                return None
            if t is not None and self.keep_retired:
                self.retired.append(t)
            t = self.buffers[which] = nt
        return t.data_ptr()

    def release_retired(self) -> None:
        self.retired.clear()


def adaptive_capacity(W: int, H: int, reset: bool = False) -> int:
    """The adaptive phase-1 capacity (tile-rect units per tile) of a W x H image on the current device; reset=True
    first returns it to its cold default."""
    v = C.c_int(0)
    check(load().dg_adaptive_capacity(int(W), int(H), 1 if reset else 0, C.byref(v)))
    return int(v.value)


def adaptive_capacity_ctx(ctx: int, W: int, H: int, reset: bool = False) -> int:
    """The same for one capacity context only (dg_adaptive_capacity_ctx)."""
    v = C.c_int(0)
    check(load().dg_adaptive_capacity_ctx(int(ctx), int(W), int(H), 1 if reset else 0, C.byref(v)))
    return int(v.value)


def release_capacity_context(ctx: int) -> None:
    """Drop a capacity context's state and device probes (dg_release_capacity_context); quiet at interpreter exit."""
    try:
        L = load()
    except Exception:  # noqa: BLE001
        return
    L.dg_release_capacity_context(int(ctx))


def capacity_contexts() -> int:
    """Capacity contexts that hold a device probe."""
    v = C.c_int(0)
    check(load().dg_capacity_contexts(C.byref(v)))
    return int(v.value)


def forward_counters(geom: torch.Tensor, P: int) -> dict:
    """The per-view counters of the last forward on a geometry buffer (dg_debug_counters; synchronises)."""
    a = (C.c_uint32 * 16)()
    check(load().dg_debug_counters(geom.data_ptr(), int(P), a, stream_of(geom.device)))
    return {"num_rendered": int(a[2]) | (int(a[3]) << 32), "e1": int(a[5]), "unfinished_tiles": int(a[6]),
            "e2": int(a[7]), "cut": bool(a[8])}


def profile_enable(on: bool = True) -> None:
    load().dg_profile_enable(1 if on else 0)


def profile_collect() -> dict[str, tuple[float, int]]:
    """{phase: (total_ms, launches)} recorded since the last collect (synchronises the recorded events)."""
    L = load()
    buf = C.create_string_buffer(8192)
    L.dg_profile_collect(buf, 8192)
    out = {}
    for item in buf.value.decode().split(";"):
        if "=" in item:
            k, v = item.split("=")
            ms, cnt = v.split("/")
            out[k] = (float(ms), int(cnt))
    return out
