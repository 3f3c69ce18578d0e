"""xerus_amd — MI355X-native implementation of xerus's dense contraction + TT-rounding hot path.

Low-level C-ABI binding: xerus_amd.capi. The product path is libxerus_amd.so (HIP kernels for
gfx950); there is no CPU fallback.
"""
from . import capi  # noqa: F401

__all__ = ["capi"]
