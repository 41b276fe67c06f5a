"""daos_amd -- MI355X-native Reed-Solomon erasure-coding engine for DAOS EC objects.

The product is libecg.so (C host layer + gfx950 HIP kernels, built from
daos_amd/csrc); `daos_amd.ecg` is its ctypes binding.  See DESIGN.md.
"""
from . import ecg  # noqa: F401

__all__ = ["ecg"]
