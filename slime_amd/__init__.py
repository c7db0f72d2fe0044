"""slime_amd — MI355X-native Reed-Solomon shard codec for encryptio/slime's internal/rs.

Layout:
  include/slime_rs.h         C-ABI (what the Go cgo shim binds)
  slime_amd/csrc/            HIP kernels for gfx950 + the C++ host library
  slime_amd/lib/             the built libslime_rs.so (in-tree)
  slime_amd.rs / .gf         Python mirror of the Go packages internal/rs, internal/rs/gf
  slime_amd.device           device-resident batch API (plans over HBM tensors)
"""
from ._native import NativeError, Panic, device_count  # noqa: F401
from . import gf, rs  # noqa: F401

__all__ = ["rs", "gf", "Panic", "NativeError", "device_count"]
