"""flashws_amd -- MI355X-native receive-path frame decode of flashws.

The product is libfws_gpu.so (HIP kernels for gfx950 behind the C ABI in
include/fws_gpu.h). This package loads it and exposes thin Python helpers for
tests and benchmarks; importing it never falls back to CPU code.
"""
from ._lib import lib, exported_symbols, FwsError, LIB_PATH  # noqa: F401

__all__ = ["lib", "exported_symbols", "FwsError", "LIB_PATH"]
