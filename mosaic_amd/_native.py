"""ctypes binding of libmosaic_hip.so (include/mosaic_hip.h).

The product path always runs through this library; there is no CPU fallback.  Loading fails
loudly (``NativeUnavailable``) when the in-tree library is missing or no GPU is visible.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmosaic_hip.so")
# A/B measurement of alternative builds (tools/): an explicit library path overrides the in-tree one
LIB_PATH = os.environ.get("MOSAIC_HIP_LIB") or LIB_PATH

MOSAIC_OK = 0
MOSAIC_E_ARG = 1
MOSAIC_E_RES = 2
MOSAIC_E_NAN = 3
MOSAIC_E_HIP = 4
MOSAIC_E_WKB = 5
MOSAIC_E_CAPACITY = 6
MOSAIC_E_NOMEM = 7

GRID_H3 = 0
GRID_BNG = 1

EXPORTS = [
    "mosaic_abi_version", "mosaic_last_error", "mosaic_init", "mosaic_destroy", "mosaic_set_option",
    "mosaic_get_stream", "mosaic_set_stream", "mosaic_sync", "mosaic_last_stats", "mosaic_last_binned_rows", "mosaic_resolution",
    "mosaic_resolution_str", "mosaic_point_to_cell", "mosaic_bng_format", "mosaic_bng_parse",
    "mosaic_chip_table_create", "mosaic_chip_table_destroy", "mosaic_chip_table_info", "mosaic_chip_table_tiles",
    "mosaic_chip_table_tile_grid", "mosaic_chip_table_raster", "mosaic_pip_join_count",
    "mosaic_pip_join_pairs", "mosaic_st_contains", "mosaic_tessellate", "mosaic_tessellate_gpu",
    "mosaic_tess_last_classify_ms", "mosaic_tess_counters", "mosaic_chip_set_info",
    "mosaic_chip_set_export", "mosaic_chip_set_columns", "mosaic_chip_set_destroy", "mosaic_kernel_times", "mosaic_last_kernel", "mosaic_point_geom_to_cell",
    "mosaic_point_geom_decode", "mosaic_intersects_aggregate",
    "mosaic_cell_kring", "mosaic_bng_format_column", "mosaic_cell_boundary_wkb", "mosaic_point_to_cell_exact",
    "mosaic_diag_libm", "mosaic_point_coords_to_cell", "mosaic_point_coords_decode", "mosaic_bng_parse_column",
    "mosaic_chip_table_create_arrow", "mosaic_chip_table_build_info", "mosaic_h3_cell_geometry",
    "mosaic_polyfill", "mosaic_cell_lists_info", "mosaic_cell_lists_export", "mosaic_cell_lists_destroy",
    "mosaic_polyfill_last_ms", "mosaic_ctx_exec", "mosaic_buffer_radius", "mosaic_chip_table_create_arrays",
    "mosaic_intersection_aggregate", "mosaic_thread_release", "mosaic_thread_count", "mosaic_stream_wait_event",
    "mosaic_intersection_aggregate_geometry", "mosaic_isect_geoms_info", "mosaic_isect_geoms_export",
    "mosaic_isect_geoms_destroy",
]

GEOM_WKB = 0
GEOM_WKT = 1
GEOM_HEX = 2
GEOM_OFFSETS32 = 0x100
ROW_NULL = 0
ROW_OK = 1
ROW_PATH = 2


class NativeUnavailable(RuntimeError):
    pass


class MosaicError(RuntimeError):
    """A non-zero mosaic_status.  ``code`` is the status; the message is the library's."""

    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


class IllegalStateException(MosaicError, ValueError):
    """Raised where the reference throws java.lang.IllegalStateException (bad resolution, NaN)."""


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", os.path.join(_HERE, "csrc")], check=True)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeUnavailable(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    # One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64.so.7 (same soname as
    # /opt/rocm's).  Whichever loads first is shared by both; if ours loads first, torch.cuda fails
    # to initialise later in the process.  So let torch load it first when torch is installed.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp, i64, i32, cp = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_char_p
    sig = {
        "mosaic_abi_version": ([], i32),
        "mosaic_last_error": ([], cp),
        "mosaic_init": ([i32, ctypes.POINTER(vp)], i32),
        "mosaic_destroy": ([vp], i32),
        "mosaic_set_option": ([vp, cp, i64], i32),
        "mosaic_get_stream": ([vp, ctypes.POINTER(vp)], i32),
        "mosaic_set_stream": ([vp, vp], i32),
        "mosaic_stream_wait_event": ([vp, vp], i32),
        "mosaic_sync": ([vp], i32),
        "mosaic_last_stats": ([vp, vp], i32),
        "mosaic_last_binned_rows": ([vp, vp], i32),
        "mosaic_resolution": ([i32, i32, ctypes.POINTER(i32)], i32),
        "mosaic_resolution_str": ([i32, cp, ctypes.POINTER(i32)], i32),
        "mosaic_point_to_cell": ([vp, i32, i32, vp, vp, vp, i64, vp, vp], i32),
        "mosaic_bng_format": ([i64, cp, ctypes.c_size_t], i32),
        "mosaic_bng_parse": ([cp, ctypes.POINTER(i64)], i32),
        "mosaic_chip_table_create": ([vp, i32, i32, i64, vp, vp, vp, vp, vp, i32, ctypes.POINTER(vp)], i32),
        "mosaic_chip_table_destroy": ([vp], i32),
        "mosaic_chip_table_info": ([vp, vp], i32),
        "mosaic_chip_table_tiles": ([vp, vp], i32),
        "mosaic_chip_table_tile_grid": ([vp, vp], i32),
        "mosaic_chip_table_raster": ([vp, vp], i32),
        "mosaic_pip_join_count": ([vp, vp, vp, vp, i64, vp], i32),
        "mosaic_pip_join_pairs": ([vp, vp, vp, vp, i64, vp, vp, i64, ctypes.POINTER(i64)], i32),
        "mosaic_st_contains": ([vp, i64, vp, vp, vp, vp, vp, i64, vp], i32),
        "mosaic_tessellate": ([i32, i32, i64, vp, vp, vp, vp, i32, i32, ctypes.POINTER(vp)], i32),
        "mosaic_chip_set_info": ([vp, ctypes.POINTER(i64), ctypes.POINTER(i64)], i32),
        "mosaic_chip_set_export": ([vp, vp, vp, vp, vp, vp], i32),
        "mosaic_chip_set_columns": ([vp, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp),
                                     ctypes.POINTER(vp)], i32),
        "mosaic_chip_set_destroy": ([vp], i32),
        "mosaic_kernel_times": ([vp, vp, i64, ctypes.POINTER(i64)], i32),
        "mosaic_last_kernel": ([vp], ctypes.c_char_p),
        "mosaic_point_geom_to_cell": ([vp, i32, i32, i32, vp, vp, vp, i64, vp, vp, ctypes.POINTER(i64)], i32),
        "mosaic_point_geom_decode": ([vp, i32, vp, vp, vp, i64, vp, vp, vp, ctypes.POINTER(i64)], i32),
        "mosaic_intersects_aggregate": ([vp, vp, vp, vp, vp, vp, i64, ctypes.POINTER(i64)], i32),
        "mosaic_cell_kring": ([vp, i32, vp, vp, i64, i32, i32, vp, vp], i32),
        "mosaic_bng_format_column": ([vp, vp, vp, i64, vp, vp, i64, ctypes.POINTER(i64)], i32),
        "mosaic_cell_boundary_wkb": ([vp, i32, vp, vp, i64, vp], i32),
        "mosaic_h3_cell_geometry": ([vp, i32, vp, vp, i64, vp, vp], i32),
        "mosaic_tessellate_gpu": ([vp, i32, i32, i64, vp, vp, vp, vp, i32, i32, ctypes.POINTER(vp)], i32),
        "mosaic_tess_last_classify_ms": ([vp], ctypes.c_double),
        "mosaic_tess_counters": ([ctypes.POINTER(i64), ctypes.POINTER(i64)], i32),
        "mosaic_point_to_cell_exact": ([vp, i32, vp, vp, i64, vp], i32),
        "mosaic_diag_libm": ([vp, i32, vp, vp, i64, vp], i32),
        "mosaic_point_coords_to_cell": ([vp, i32, i32, vp, vp, vp, vp, vp, vp, i64, vp, vp, ctypes.POINTER(i64)], i32),
        "mosaic_point_coords_decode": ([vp, vp, vp, vp, vp, vp, vp, i64, vp, vp, vp, ctypes.POINTER(i64)], i32),
        "mosaic_bng_parse_column": ([vp, i32, vp, vp, vp, i64, vp], i32),
        "mosaic_chip_table_create_arrow": ([vp, i32, i32, i64, vp, vp, vp, i32, vp, vp, i32, ctypes.POINTER(vp)], i32),
        "mosaic_chip_table_build_info": ([vp, vp, vp], i32),
        "mosaic_polyfill": ([vp, i32, i32, i64, vp, vp, vp, vp, ctypes.POINTER(vp)], i32),
        "mosaic_cell_lists_info": ([vp, ctypes.POINTER(i64), ctypes.POINTER(i64)], i32),
        "mosaic_cell_lists_export": ([vp, vp, vp, vp], i32),
        "mosaic_cell_lists_destroy": ([vp], i32),
        "mosaic_polyfill_last_ms": ([], ctypes.c_double),
        "mosaic_buffer_radius": ([vp, i32, i32, i64, vp, vp, vp, vp, vp], i32),
        "mosaic_chip_table_create_arrays": ([vp, i32, i32, i32, vp, vp, vp, vp, vp, ctypes.POINTER(vp)], i32),
        "mosaic_intersection_aggregate": ([vp, vp, vp, vp, vp, vp, vp, i64, ctypes.POINTER(i64)], i32),
        "mosaic_intersection_aggregate_geometry": ([vp, vp, vp, ctypes.POINTER(vp)], i32),
        "mosaic_isect_geoms_info": ([vp, ctypes.POINTER(i64), ctypes.POINTER(i64)], i32),
        "mosaic_isect_geoms_export": ([vp, vp, vp, vp, vp, vp, vp], i32),
        "mosaic_isect_geoms_destroy": ([vp], i32),
        "mosaic_thread_release": ([vp], i32),
        "mosaic_thread_count": ([vp, ctypes.POINTER(i64), ctypes.POINTER(i64)], i32),
        "mosaic_ctx_exec": ([vp, ctypes.POINTER(i32), ctypes.POINTER(vp), ctypes.POINTER(i32), ctypes.POINTER(i32)],
                            i32),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def check(rc):
    if rc == MOSAIC_OK:
        return
    msg = lib().mosaic_last_error().decode(errors="replace")
    if rc in (MOSAIC_E_RES, MOSAIC_E_NAN):
        raise IllegalStateException(rc, msg)
    raise MosaicError(rc, msg)


def ptr(a):
    """Address of a numpy array or a torch tensor (host or device)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    raise TypeError(f"unsupported buffer type {type(a)}")
