"""Import-path shim: `from fused_ssim import fused_ssim` resolves to the MI355X implementation."""
from dogs_amd.fused_ssim import *  # noqa: F401,F403
