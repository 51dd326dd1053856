"""mosaic_amd: MI355X-native engine for Mosaic's point-in-polygon chip-join hot path.

Product path: libmosaic_hip.so (mosaic_amd/csrc, HIP for gfx950) behind the C ABI in
include/mosaic_hip.h; this package is the host-side mirror of the reference's function surface.
"""
from ._native import IllegalStateException, MosaicError, NativeUnavailable  # noqa: F401
from .context import BNGIndexSystem, ChipTable, H3IndexSystem, MosaicContext, RowPathRequired  # noqa: F401

__all__ = ["MosaicContext", "ChipTable", "H3IndexSystem", "BNGIndexSystem", "IllegalStateException",
           "MosaicError", "NativeUnavailable"]
