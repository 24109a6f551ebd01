"""The drop-in boundary without a GPU: libdogs_hip.so builds for gfx950 (hipcc cross-compiles here), loads, and
exports every entry point include/dogs_hip.h declares; the Python surface keeps the reference's names and
error behaviour (diff_gaussian_rasterization/__init__.py:236-260, rasterize_points.cu:78-80) and refuses to run
on anything but a HIP device -- there is no CPU fallback."""
import ctypes as C
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dogs_hip.h")


@pytest.fixture(scope="module")
def lib_path():
    from dogs_amd import _lib
    from dogs_amd import build as B
    if not os.path.exists(_lib.LIB_PATH):
        B.build()
    return _lib.LIB_PATH


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    return sorted(set(re.findall(r"\b(dg_[a-z0-9_]+)\s*\(", text)) - {"dg_alloc_fn"})


def test_header_declares_the_reference_surface():
    names = header_functions()
    for n in ("dg_rasterize_forward", "dg_rasterize_backward", "dg_mark_visible", "dg_rasterize_filter",
              "dg_adam_update", "dg_fused_ssim_forward", "dg_fused_ssim_backward", "dg_dist_cuda2", "dg_last_error"):
        assert n in names


def test_library_exports_every_declared_symbol(lib_path):
    L = C.CDLL(lib_path)
    missing = [n for n in header_functions() if not hasattr(L, n)]
    assert not missing, f"declared in dogs_hip.h but not exported: {missing}"
    from dogs_amd import _lib
    assert set(_lib.EXPORTS) <= set(header_functions())


def test_library_is_gfx950_code_object(lib_path):
    blob = open(lib_path, "rb").read()
    assert b"gfx950" in blob


def test_version_and_last_error(lib_path):
    from dogs_amd import _lib
    L = _lib.load()
    assert L.dg_version() >= 1
    assert isinstance(L.dg_last_error(), (bytes, type(None)))


def test_python_surface_names():
    import diff_gaussian_rasterization as d
    import fused_ssim
    from simple_knn._C import distCUDA2  # noqa: F401
    for n in ("GaussianRasterizationSettings", "GaussianRasterizer", "SparseGaussianAdam", "rasterize_gaussians"):
        assert hasattr(d, n)
    assert hasattr(fused_ssim, "fused_ssim")
    from diff_gaussian_rasterization import _C
    for n in ("rasterize_gaussians", "rasterize_gaussians_backward", "mark_visible", "rasterize_gaussians_filter",
              "adamUpdate", "fusedssim", "fusedssim_backward"):
        assert hasattr(_C, n)


def _settings(dev="cpu"):
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    return GaussianRasterizationSettings(image_height=48, image_width=64, tanfovx=0.5, tanfovy=0.4,
                                         bg=torch.zeros(3), scale_modifier=1.0, viewmatrix=torch.eye(4),
                                         projmatrix=torch.eye(4), sh_degree=3, campos=torch.zeros(3),
                                         prefiltered=False, debug=False, antialiasing=False,
                                         depth_threshold=0.0)


def test_rasterizer_argument_errors_match_reference():
    from diff_gaussian_rasterization import GaussianRasterizer
    r = GaussianRasterizer(_settings())
    m = torch.zeros(4, 3)
    o = torch.ones(4, 1)
    with pytest.raises(Exception, match="exactly one of either SHs|excatly one of either SHs"):
        r(m, m, o, shs=torch.zeros(4, 15, 3), colors_precomp=torch.zeros(4, 3), scales=m, rotations=torch.zeros(4, 4))
    with pytest.raises(Exception, match="scale/rotation pair or precomputed 3D covariance"):
        r(m, m, o, colors_precomp=torch.zeros(4, 3))


def test_no_cpu_fallback():
    """CPU tensors must raise (RuntimeError), never silently compute on the host."""
    from diff_gaussian_rasterization import _C
    e = torch.empty(0)
    with pytest.raises((RuntimeError, ImportError)):
        _C.rasterize_gaussians(torch.zeros(3), torch.zeros(4, 3), e, torch.ones(4, 1), torch.ones(4, 3),
                               torch.ones(4, 4), 1.0, e, torch.eye(4), torch.eye(4), 0.5, 0.4, 48, 64,
                               torch.zeros(4, 1, 3), torch.zeros(4, 15, 3), 3, torch.zeros(3), False, False, False)


def test_ctypes_structs_match_the_header(tmp_path):
    """sizeof/offsetof of the C structs (gcc on include/dogs_hip.h) equal the ctypes mirrors in dogs_amd/_lib.py."""
    import shutil
    import subprocess
    from dogs_amd import _lib
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    checks = {
        "dg_raster_args": (_lib.DgRasterArgs, ["P", "prefix_per_tile", "scale_modifier", "bg", "campos"]),
        "dg_adam_group": (_lib.DgAdamGroup, ["param", "lr", "eps", "M"]),
        "dg_densify_stats": (_lib.DgDensifyStats, ["radii", "dmeans2D_stride", "max_radii2D", "denom"]),
        "dg_gaussian_set": (_lib.DgGaussianSet, ["N", "params", "exp_avg_sq", "width", "grad_accum", "denom"]),
        "dg_densify_args": (_lib.DgDensifyArgs, ["set", "max_grad", "replicas", "big_extent", "samples",
                                                 "out_params", "out_exp_avg_sq", "state", "state2", "nc", "n_out"]),
    }
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for s, (_, fields) in checks.items():
        lines.append(f'printf("{s} %zu\\n", sizeof({s}));')
        for f in fields:
            lines.append(f'printf("{s}.{f} %zu\\n", offsetof({s}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", str(src), "-o", str(exe)], check=True)
    got = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                       check=True).stdout.split("\n") if l)
    for s, (cls, fields) in checks.items():
        assert int(got[s]) == C.sizeof(cls), s
        for f in fields:
            assert int(got[f"{s}.{f}"]) == getattr(cls, f).offset, f"{s}.{f}"


def test_tensor_arena_bucket_sizes():
    """TensorArena rounds per-view buffer requests up (caching-allocator reuse): at most 12.5% more above 1 MiB,
    exact below, monotone, and a multiple of an eighth of the request's power of two."""
    from dogs_amd._lib import _bucket
    prev = 0
    for n in [1, 17, 4096, 1 << 20, (1 << 20) + 1, 3_000_000, 50_000_123, 123_456_789, (1 << 31) + 5]:
        b = _bucket(n)
        assert b >= n and b >= prev
        prev = b
        if n <= 1 << 20:
            assert b == n
        else:
            assert b <= n * 1.125 and b % (1 << (n.bit_length() - 4)) == 0
