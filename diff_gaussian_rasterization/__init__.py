"""Import-path shim: `from diff_gaussian_rasterization import ...` resolves to the MI355X implementation."""
from dogs_amd.diff_gaussian_rasterization import *  # noqa: F401,F403
from dogs_amd.diff_gaussian_rasterization import _C, _RasterizeGaussians, cpu_deep_copy_tuple  # noqa: F401
