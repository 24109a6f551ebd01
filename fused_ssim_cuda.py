"""Import-path shim for the reference's `fused_ssim_cuda` extension module."""
from dogs_amd.fused_ssim._cuda import fusedssim, fusedssim_backward  # noqa: F401
