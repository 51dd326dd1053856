"""Host-side mirror of the reference's function surface for the PIP chip-join path.

Mirrors (bransonf/mosaic 0.3.9, src/main/scala/com/databricks/labs/mosaic/):
  * ``MosaicContext.build(indexSystem, geometryAPI)``       functions/MosaicContext.scala:796-800
  * ``functions.grid_pointascellid / grid_longlatascellid``  MosaicContext.scala:655-668
  * ``functions.st_contains``                                MosaicContext.scala (st_contains) ->
                                                             expressions/geometry/ST_Contains.scala:21-64
  * ``H3IndexSystem / BNGIndexSystem.getResolution``         core/index/H3IndexSystem.scala:39-54,
                                                             core/index/BNGIndexSystem.scala:342-353
  * the chip join of the Quickstart                         notebooks/examples/python/QuickstartNotebook.py:205-219,
                                                             sql/join/PointInPolygonJoin.scala:68-84
Everything computes on the GPU through libmosaic_hip.so; inputs are columnar (numpy arrays or torch
tensors, host or device), the Spark row wrappers are not reproduced.  Errors follow the reference:
bad resolutions and NaN BNG coordinates raise ``IllegalStateException`` with the reference's message.
"""
import ctypes
import threading

import numpy as np

from . import _native as N
from . import wkb as W


class IndexSystem:
    name = None
    grid = None
    cell_id_type = "long"

    def get_resolution(self, res):
        raise NotImplementedError


class H3IndexSystem(IndexSystem):
    """core/index/H3IndexSystem.scala; cell ids are LongType."""

    name = "H3"
    grid = N.GRID_H3
    cell_id_type = "long"

    def get_resolution(self, res):
        out = ctypes.c_int(0)
        if isinstance(res, (bool,)):
            raise ValueError("Resolution must be an Int or String.")
        if isinstance(res, (int, np.integer)):
            N.check(N.lib().mosaic_resolution(self.grid, int(res), ctypes.byref(out)))
        elif isinstance(res, str):
            N.check(N.lib().mosaic_resolution_str(self.grid, res.encode(), ctypes.byref(out)))
        else:
            raise ValueError("Resolution must be an Int or String.")
        return out.value

    def format(self, cell_id):
        return format(int(cell_id), "x")

    def parse(self, s):
        return int(s, 16)


class BNGIndexSystem(IndexSystem):
    """core/index/BNGIndexSystem.scala; cell ids default to StringType (MosaicContext.scala:41-48)."""

    name = "BNG"
    grid = N.GRID_BNG
    cell_id_type = "string"

    def get_resolution(self, res):
        out = ctypes.c_int(0)
        if isinstance(res, (int, np.integer)) and not isinstance(res, bool):
            N.check(N.lib().mosaic_resolution(self.grid, int(res), ctypes.byref(out)))
        elif isinstance(res, str):
            N.check(N.lib().mosaic_resolution_str(self.grid, res.encode(), ctypes.byref(out)))
        else:
            raise N.IllegalStateException(N.MOSAIC_E_RES, f"BNG resolution not supported; found {res}")
        return out.value

    def format(self, cell_id):
        buf = ctypes.create_string_buffer(64)
        rc = N.lib().mosaic_bng_format(int(cell_id), buf, 64)
        if rc < 0 or rc > 64:
            N.check(rc if rc > 0 else N.MOSAIC_E_ARG)
        return buf.value.decode()

    def parse(self, s):
        out = ctypes.c_int64(0)
        N.check(N.lib().mosaic_bng_parse(s.encode(), ctypes.byref(out)))
        return out.value


INDEX_SYSTEMS = {"H3": H3IndexSystem, "BNG": BNGIndexSystem}


def _f64(a):
    """Contiguous float64 buffer (numpy or torch, host or device) kept alive by the caller."""
    if hasattr(a, "data_ptr"):
        import torch

        if a.dtype != torch.float64:
            a = a.to(torch.float64)
        return a.contiguous()
    return np.ascontiguousarray(a, dtype=np.float64)


def _is_torch(a):
    return hasattr(a, "data_ptr") and not isinstance(a, np.ndarray)


class RowPathRequired(RuntimeError):
    """Rows the engine leaves to the reference's row-wise expression (MOSAIC_ROW_PATH): geometry
    types other than Point (the reference indexes their centroid), POINT EMPTY and malformed rows
    (on which the reference throws).  ``rows`` holds their indices.  The columnar exec of
    INTEGRATION.md evaluates them with PointIndexGeom.nullSafeEval; this mirror reports them."""

    def __init__(self, rows):
        super().__init__(f"{len(rows)} row(s) need the reference row path (first: row {int(rows[0])})")
        self.rows = rows


def geometry_column(geoms):
    """A sequence of WKB (bytes) / WKT (str) / hex-WKB (str with format="hex") rows, None = null,
    as an Arrow-layout column: (format, int64 offsets[n+1], uint8 values, uint8 validity or None)."""
    geoms = list(geoms)
    kinds = {type(g) for g in geoms if g is not None}
    if kinds <= {bytes, bytearray, memoryview}:
        fmt = N.GEOM_WKB
        rows = [bytes(g) if g is not None else b"" for g in geoms]
    elif kinds <= {str}:
        fmt = N.GEOM_WKT
        rows = [g.encode("utf-8") if g is not None else b"" for g in geoms]
    else:
        raise TypeError("a geometry column holds WKB bytes or WKT strings")
    lens = np.fromiter((len(r) for r in rows), np.int64, len(rows))
    offsets = np.zeros(len(rows) + 1, np.int64)
    np.cumsum(lens, out=offsets[1:])
    data = np.frombuffer(b"".join(rows), np.uint8) if offsets[-1] else np.zeros(1, np.uint8)
    valid = None
    if any(g is None for g in geoms):
        valid = np.fromiter((g is not None for g in geoms), np.uint8, len(geoms))
    return fmt, offsets, data, valid


class CoordsColumn:
    """The COORDS geometry form (InternalGeometryType: struct<typeId, srid, boundaries:
    array<array<array<double>>>, holes: array<array<array<array<double>>>>>,
    core/types/model/InternalGeometry.scala) as Arrow columns: type_id int32[n], srid int32[n],
    boundary_offsets int32[n + 1] (row -> boundaries), coord_offsets int32 (boundary -> coordinates),
    value_offsets int32 (coordinate -> values), values float64, validity uint8 or None.  The holes
    column is not kept (no point has one)."""

    def __init__(self, type_id, srid, boundary_offsets, coord_offsets, value_offsets, values, valid=None):
        self.type_id = np.ascontiguousarray(type_id, np.int32)
        self.srid = np.ascontiguousarray(srid, np.int32)
        self.boundary_offsets = np.ascontiguousarray(boundary_offsets, np.int32)
        self.coord_offsets = np.ascontiguousarray(coord_offsets, np.int32)
        self.value_offsets = np.ascontiguousarray(value_offsets, np.int32)
        self.values = np.ascontiguousarray(values, np.float64)
        self.valid = None if valid is None else np.ascontiguousarray(valid, np.uint8)

    def __len__(self):
        return len(self.type_id)

    @classmethod
    def from_rows(cls, rows):
        """rows: (type_id, srid, boundaries, holes) tuples -- boundaries a list of coordinate lists,
        a coordinate a list of 2 or 3 floats -- or None for a null row."""
        tid, srid, bo, co, vo, vals, valid = [], [], [0], [0], [0], [], []
        for r in rows:
            valid.append(r is not None)
            t, sr, bnds = (r[0], r[1], r[2]) if r is not None else (0, 0, [])
            tid.append(t)
            srid.append(sr)
            for b in bnds:
                for c in b:
                    vals.extend(float(v) for v in c)
                    vo.append(len(vals))
                co.append(len(vo) - 1)
            bo.append(len(co) - 1)
        return cls(tid, srid, bo, co, vo, vals, np.array(valid, np.uint8))


def st_point(x, y):
    """ST_Point (expressions/constructors/ST_Point.scala:27-32): InternalGeometry(POINT, 0,
    [[[x, y]]], [[]]) per row, as a CoordsColumn."""
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    n = len(x)
    vals = np.empty(2 * n, np.float64)
    vals[0::2] = x
    vals[1::2] = y
    ar = np.arange(n + 1, dtype=np.int32)
    return CoordsColumn(np.ones(n, np.int32), np.zeros(n, np.int32), ar, ar, 2 * ar, vals)


def _is_arrow_utf8(v):
    """An Arrow utf8 column given explicitly as (offsets int32 / int64 array, chars bytes / uint8 array)."""
    if not (isinstance(v, tuple) and len(v) == 2):
        return False
    offs, chars = v
    return (isinstance(offs, np.ndarray) and offs.dtype in (np.int32, np.int64) and
            (isinstance(chars, (bytes, bytearray)) or (isinstance(chars, np.ndarray) and chars.dtype == np.uint8)))


def _points_xy(points):
    """Accepts (x, y) arrays or an (n, 2) array (host or device)."""
    if isinstance(points, tuple) and len(points) == 2:
        return _f64(points[0]), _f64(points[1])
    if isinstance(points, np.ndarray) and points.ndim == 2 and points.shape[1] == 2:
        return _f64(points[:, 0]), _f64(points[:, 1])
    if _is_torch(points) and points.dim() == 2:
        return _f64(points[:, 0]), _f64(points[:, 1])
    return None


class ChipTable:
    """Device-resident build side of the chip join: rows of ChipType(is_core, index_id, wkb) plus the
    key of the polygon each chip belongs to (core/types/ChipType.scala:17-28)."""

    def __init__(self, ctx, is_core, index_id, wkb_list, polygon_key, n_polygons=None):
        self.ctx = ctx
        is_core = np.ascontiguousarray(is_core, dtype=np.uint8)
        strings = not _is_arrow_utf8(index_id) and len(index_id) and isinstance(index_id[0], str)
        if ctx.index_system.cell_id_type == "string" and (_is_arrow_utf8(index_id) or strings):
            # StringType ids (the BNG default, BNGIndexSystem.scala:28): parsed on the GPU
            index_id = ctx.bng_parse_column(index_id)
        elif strings:
            # string ids of a LongType index system (H3 hex strings, H3IndexSystem.parse)
            index_id = [ctx.index_system.parse(v) for v in index_id]
        elif _is_arrow_utf8(index_id):
            raise ValueError(f"an Arrow utf8 id column needs a StringType index system, not {ctx.index_system.name}")
        index_id = np.ascontiguousarray(index_id, dtype=np.int64)
        polygon_key = np.ascontiguousarray(polygon_key, dtype=np.int32)
        if isinstance(wkb_list, tuple) and len(wkb_list) == 2:
            # Arrow binary (int32 offsets) or large_binary (int64)
            offsets = np.ascontiguousarray(wkb_list[0])
            if offsets.dtype != np.int32:
                offsets = offsets.astype(np.int64, copy=False)
            data = np.ascontiguousarray(wkb_list[1], dtype=np.uint8)
        else:
            lens = np.array([0 if w is None else len(w) for w in wkb_list], dtype=np.int64)
            offsets = np.zeros(len(lens) + 1, np.int64)
            np.cumsum(lens, out=offsets[1:])
            data = np.frombuffer(b"".join(b"" if w is None else bytes(w) for w in wkb_list), dtype=np.uint8)
            data = np.ascontiguousarray(data) if len(data) else np.zeros(1, np.uint8)
        n = len(index_id)
        if not (len(is_core) == n == len(polygon_key) == len(offsets) - 1):
            raise ValueError("chip columns have different lengths")
        if n_polygons is None:
            n_polygons = int(polygon_key.max()) + 1 if n else 0
        self.n_polygons = int(n_polygons)
        self.n_chips = n
        h = ctypes.c_void_p()
        N.check(N.lib().mosaic_chip_table_create_arrow(
            ctx.handle, ctx.index_system.grid, ctx.resolution_of_table, n, N.ptr(is_core), N.ptr(index_id),
            N.ptr(offsets), 1 if offsets.dtype == np.int32 else 0, N.ptr(data), N.ptr(polygon_key), self.n_polygons,
            ctypes.byref(h)))
        self.handle = h

    @classmethod
    def from_arrays(cls, ctx, chip_offsets, is_core, index_id, wkb_list):
        """The array form of the build side (PointInPolygonJoin.joinArrayRows,
        sql/join/PointInPolygonJoin.scala:39-66): polygon row p's chip array (grid_tessellate output)
        is rows [chip_offsets[p], chip_offsets[p + 1]) of the flattened chip columns; a point joins a
        row at most once, through the row's first chip with the point's cell."""
        self = cls.__new__(cls)
        self.ctx = ctx
        chip_offsets = np.ascontiguousarray(chip_offsets, dtype=np.int64)
        is_core = np.ascontiguousarray(is_core, dtype=np.uint8)
        index_id = np.ascontiguousarray(index_id, dtype=np.int64)
        lens = np.array([0 if w is None else len(w) for w in wkb_list], dtype=np.int64)
        offsets = np.zeros(len(lens) + 1, np.int64)
        np.cumsum(lens, out=offsets[1:])
        data = np.frombuffer(b"".join(b"" if w is None else bytes(w) for w in wkb_list), dtype=np.uint8)
        data = np.ascontiguousarray(data) if len(data) else np.zeros(1, np.uint8)
        self.n_polygons = len(chip_offsets) - 1
        self.n_chips = len(index_id)
        h = ctypes.c_void_p()
        N.check(N.lib().mosaic_chip_table_create_arrays(
            ctx.handle, ctx.index_system.grid, ctx.resolution_of_table, self.n_polygons, N.ptr(chip_offsets),
            N.ptr(is_core), N.ptr(index_id), N.ptr(offsets), N.ptr(data), ctypes.byref(h)))
        self.handle = h
        return self

    def info(self):
        out = np.zeros(8, np.int64)
        N.check(N.lib().mosaic_chip_table_info(self.handle, N.ptr(out)))
        keys = ["n_chips", "n_cells", "n_border", "n_vertices", "n_rings", "device_bytes", "hash_capacity",
                "n_polygons"]
        return dict(zip(keys, (int(v) for v in out)))

    def tiles(self):
        """The H3 tile directory of this table (tiles.h): whether it was built, and its size."""
        out = np.zeros(13, np.int64)
        N.check(N.lib().mosaic_chip_table_tiles(self.handle, N.ptr(out)))
        keys = ["built", "nx", "ny", "records", "entries", "full_tiles", "rings", "raster", "raster_sub",
                "raster_cell", "pure_sub_blocks", "mixed_sub_blocks", "mixed_cells"]
        d = dict(zip(keys, (int(v) for v in out)))
        g = np.zeros(4, np.float64)
        N.check(N.lib().mosaic_chip_table_tile_grid(self.handle, N.ptr(g)))
        d.update(x0=float(g[0]), y0=float(g[1]), sx=float(g[2]), sy=float(g[3]))
        r = np.zeros(9, np.int64)
        N.check(N.lib().mosaic_chip_table_raster(self.handle, N.ptr(r)))
        d.update(line_sub_blocks=int(r[0]), quad_entries=int(r[1]), quad_shift=int(r[2]), raster_bytes=int(r[3]),
                 stream=int(r[4]), image_records=int(r[5]), image_bytes=int(r[6]), image_max_bytes=int(r[7]),
                 leaf_lines=int(r[8]))
        return d

    def build_info(self):
        """Build cost of this table in ms (chip core, tile directory, point-raster classification,
        point-raster assembly) and the point raster's FNV-1a digest (0: no raster)."""
        ms = np.zeros(4, np.float64)
        dig = np.zeros(1, np.uint64)
        N.check(N.lib().mosaic_chip_table_build_info(self.handle, N.ptr(ms), N.ptr(dig)))
        return dict(core_ms=float(ms[0]), directory_ms=float(ms[1]), raster_classify_ms=float(ms[2]),
                    raster_assemble_ms=float(ms[3]), raster_digest=int(dig[0]))

    def close(self):
        if self.handle:
            N.lib().mosaic_chip_table_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MosaicContext:
    """``MosaicContext.build(indexSystem, geometryAPI)``; geometry API is JTS semantics only."""

    def __init__(self, index_system="H3", geometry_api="JTS", device=0, jdk=8):
        if geometry_api.upper() != "JTS":
            raise ValueError("only JTS semantics are implemented (BASELINE north_star)")
        if index_system not in INDEX_SYSTEMS:
            raise ValueError(f"unsupported index system {index_system} (H3, BNG)")
        self.index_system = INDEX_SYSTEMS[index_system]()
        self.geometry_api = "JTS"
        h = ctypes.c_void_p()
        N.check(N.lib().mosaic_init(int(device), ctypes.byref(h)))
        self.handle = h
        self.device = device
        self.set_option("jdk", jdk)
        self.resolution_of_table = None
        self._bound = threading.local()  # per calling thread: the stream set with set_stream

    @classmethod
    def build(cls, index_system="H3", geometry_api="JTS", device=0, jdk=8):
        return cls(index_system, geometry_api, device, jdk)

    def set_option(self, key, value):
        N.check(N.lib().mosaic_set_option(self.handle, key.encode(), int(value)))

    def stream(self):
        s = ctypes.c_void_p()
        N.check(N.lib().mosaic_get_stream(self.handle, ctypes.byref(s)))
        return s.value

    def set_stream(self, stream_handle):
        N.check(N.lib().mosaic_set_stream(self.handle, stream_handle))
        # a null handle binds no caller stream of ours to order against (HIP's null stream)
        self._bound.stream = stream_handle or None

    def wait_event(self, event_handle):
        """Order this thread's later calls after a recorded hipEvent_t (mosaic_stream_wait_event)."""
        N.check(N.lib().mosaic_stream_wait_event(self.handle, event_handle))

    def _order(self, *arrays):
        """Device columns written on torch's current stream are complete before the engine's own
        (non-blocking) stream reads them: without a stream bound with set_stream, an event recorded
        on torch's current stream is waited for on the engine's stream (no host block); a bound
        stream orders the work itself."""
        if getattr(self._bound, "stream", None) is not None:
            return
        for a in arrays:
            if _is_torch(a) and a.is_cuda:
                import torch

                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(a.device))
                self.wait_event(ev.cuda_event)
                self._bound.last_event = ev  # kept alive until the next ordered call
                return

    def sync(self):
        N.check(N.lib().mosaic_sync(self.handle))

    def last_kernel(self):
        """name of the dominant kernel of this thread's last join call (mosaic_last_kernel)"""
        return N.lib().mosaic_last_kernel(self.handle).decode()

    def kernel_times(self, cap=4096):
        """Elapsed ms of each fused join kernel since option "timing" was set (HIP events)."""
        out = np.zeros(cap, np.float64)
        n = ctypes.c_int64(0)
        N.check(N.lib().mosaic_kernel_times(self.handle, N.ptr(out), cap, ctypes.byref(n)))
        return out[:min(n.value, cap)]

    def thread_release(self):
        """Free the calling thread's execution state on this context (its stream, scratch, events);
        a later call from the thread creates a fresh one (mosaic_thread_release)."""
        N.check(N.lib().mosaic_thread_release(self.handle))
        # the released state's stream binding is gone: later calls run on a fresh context stream
        self._bound.stream = None

    def thread_states(self):
        """(live per-thread states, scratch bytes they hold) (mosaic_thread_count)."""
        n, b = ctypes.c_int64(0), ctypes.c_int64(0)
        N.check(N.lib().mosaic_thread_count(self.handle, ctypes.byref(n), ctypes.byref(b)))
        return n.value, b.value

    def last_binned_rows(self):
        """Rows the last join on this thread sorted on its binned path (0: another path)."""
        out = np.zeros(1, np.int64)
        N.check(N.lib().mosaic_last_binned_rows(self.handle, N.ptr(out)))
        return int(out[0])

    def last_stats(self):
        out = np.zeros(3, np.int64)
        N.check(N.lib().mosaic_last_stats(self.handle, N.ptr(out)))
        return {"exact_path_rows": int(out[0]), "contains_tests": int(out[1]), "pairs": int(out[2])}

    def close(self):
        if getattr(self, "handle", None):
            N.lib().mosaic_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- grid functions ----
    def _cells(self, x, y, resolution, valid=None):
        res = self.index_system.get_resolution(resolution)
        x, y = _f64(x), _f64(y)
        self._order(x, y, valid)
        n = int(x.shape[0])
        if _is_torch(x):
            import torch

            out = torch.empty(n, dtype=torch.int64, device=x.device)
        else:
            out = np.empty(n, np.int64)
        v = None if valid is None else np.ascontiguousarray(valid, dtype=np.uint8)
        ov = None if v is None else np.empty(n, np.uint8)
        N.check(N.lib().mosaic_point_to_cell(self.handle, self.index_system.grid, res, N.ptr(x), N.ptr(y), N.ptr(v), n,
                                             N.ptr(out), N.ptr(ov)))
        return (out, ov) if v is not None else out

    def _serialize(self, cells):
        """IndexSystem.serializeCellId: Long for H3, String for BNG (IndexSystem.scala:37-46)."""
        if self.index_system.cell_id_type == "string":
            offs, chars = self.bng_format_column(cells)
            return [chars[offs[i]:offs[i + 1]].decode() for i in range(len(offs) - 1)]
        return cells

    def bng_format_column(self, cells, valid=None):
        """BNG ids -> Arrow utf8 column (int64 offsets[n + 1], bytes), formatted on the GPU
        (BNGIndexSystem.format, BNGIndexSystem.scala:114-129)."""
        ids = cells.contiguous() if _is_torch(cells) else np.ascontiguousarray(cells, np.int64)
        self._order(ids, valid)
        n = int(ids.shape[0])
        offs = np.zeros(n + 1, np.int64)
        need = ctypes.c_int64(0)
        v = None if valid is None else np.ascontiguousarray(valid, np.uint8)
        cap = 16 * n
        chars = np.zeros(max(cap, 1), np.uint8)
        N.check(N.lib().mosaic_bng_format_column(self.handle, N.ptr(ids), None if v is None else N.ptr(v), n,
                                                 N.ptr(offs), N.ptr(chars), cap, ctypes.byref(need)))
        return offs, chars[:need.value].tobytes()

    def bng_parse_column(self, strings, valid=None):
        """BNG string ids -> long ids, parsed on the GPU (BNGIndexSystem.parse,
        BNGIndexSystem.scala:391-413).  ``strings``: a sequence of str (None = null) or an Arrow utf8
        tuple (offsets int32 / int64, chars)."""
        if _is_arrow_utf8(strings):
            offs, chars = strings
            offs = np.ascontiguousarray(offs)
            chars = np.frombuffer(chars, np.uint8) if isinstance(chars, (bytes, bytearray)) else np.ascontiguousarray(chars, np.uint8)
        else:
            enc = [b"" if v is None else v.encode() for v in strings]
            if valid is None and any(v is None for v in strings):
                valid = np.array([v is not None for v in strings], np.uint8)
            offs = np.zeros(len(enc) + 1, np.int32)
            np.cumsum([len(e) for e in enc], out=offs[1:])
            chars = np.frombuffer(b"".join(enc) or b"\0", np.uint8)
        o32 = 1 if offs.dtype == np.int32 else 0
        if not o32:
            offs = offs.astype(np.int64, copy=False)
        n = len(offs) - 1
        out = np.zeros(max(n, 1), np.int64)
        v = None if valid is None else np.ascontiguousarray(valid, np.uint8)
        N.check(N.lib().mosaic_bng_parse_column(self.handle, o32, N.ptr(offs), N.ptr(chars), N.ptr(v), n, N.ptr(out)))
        return out[:n]

    def grid_longlatascellid(self, lon, lat, resolution, raw=False):
        """PointIndexLonLat (expressions/index/PointIndexLonLat.scala:44-51)."""
        cells = self._cells(lon, lat, resolution)
        return cells if raw else self._serialize(cells)

    def grid_pointascellid(self, points, resolution, raw=False, fmt=None, return_status=False):
        """PointIndexGeom (expressions/index/PointIndexGeom.scala:32-40).  ``points``: (x, y)
        arrays / an (n, 2) array, or a geometry column -- a sequence of WKB bytes / WKT strings
        (None = null) or an Arrow-layout tuple (offsets, values, validity) with ``fmt`` one of
        "wkb" / "wkt" / "hex" -- decoded on the device (mosaic_point_geom_to_cell).  Rows the
        engine leaves to the reference row path raise RowPathRequired unless return_status, which
        returns (cells, row_status) with row_status 0 null / 1 ok / 2 row path."""
        xy = _points_xy(points)
        if xy is not None:
            cells = self._cells(xy[0], xy[1], resolution)
            return cells if raw else self._serialize(cells)
        res = self.index_system.get_resolution(resolution)
        if isinstance(points, CoordsColumn):
            n = len(points)
            out = np.empty(n, np.int64)
            status = np.empty(n, np.uint8)
            n_rp = ctypes.c_int64(0)
            N.check(N.lib().mosaic_point_coords_to_cell(
                self.handle, self.index_system.grid, res, N.ptr(points.type_id), N.ptr(points.boundary_offsets),
                N.ptr(points.coord_offsets), N.ptr(points.value_offsets),
                N.ptr(points.values) if len(points.values) else None, N.ptr(points.valid), n, N.ptr(out),
                N.ptr(status), ctypes.byref(n_rp)))
            if n_rp.value and not return_status:
                raise RowPathRequired(np.flatnonzero(status == N.ROW_PATH))
            cells = out if raw else self._serialize(out)
            return (cells, status) if return_status else cells
        if isinstance(points, tuple) and len(points) == 3:
            offsets, data, valid = points
            f = {"wkb": N.GEOM_WKB, "wkt": N.GEOM_WKT, "hex": N.GEOM_HEX}[fmt or "wkb"]
        else:
            f, offsets, data, valid = geometry_column(points)
            if fmt == "hex":
                f = N.GEOM_HEX
        if not _is_torch(offsets):
            offsets = np.ascontiguousarray(offsets)
            if offsets.dtype == np.int32:
                f |= N.GEOM_OFFSETS32
            else:
                offsets = offsets.astype(np.int64, copy=False)
        elif str(offsets.dtype) == "torch.int32":
            f |= N.GEOM_OFFSETS32
        if valid is not None and not _is_torch(valid):
            valid = np.ascontiguousarray(valid, dtype=np.uint8)
        n = int(offsets.shape[0]) - 1
        self._order(offsets, data, valid)
        if _is_torch(offsets):
            import torch

            out = torch.empty(n, dtype=torch.int64, device=offsets.device)
            status = torch.empty(n, dtype=torch.uint8, device=offsets.device)
        else:
            out = np.empty(n, np.int64)
            status = np.empty(n, np.uint8)
        n_rp = ctypes.c_int64(0)
        N.check(N.lib().mosaic_point_geom_to_cell(self.handle, self.index_system.grid, res, f, N.ptr(offsets),
                                                  N.ptr(data), N.ptr(valid), n, N.ptr(out), N.ptr(status),
                                                  ctypes.byref(n_rp)))
        if n_rp.value and not return_status:
            st = status.cpu().numpy() if _is_torch(status) else status
            raise RowPathRequired(np.flatnonzero(st == N.ROW_PATH))
        cells = out if raw else self._serialize(out)
        return (cells, status) if return_status else cells

    def decode_points(self, points, fmt=None):
        """Point geometry column (as in grid_pointascellid) -> (x, y) on the device decoder
        (mosaic_point_geom_decode); raises RowPathRequired for rows it does not decode."""
        if isinstance(points, tuple) and len(points) == 3:
            offsets, data, valid = points
            f = {"wkb": N.GEOM_WKB, "wkt": N.GEOM_WKT, "hex": N.GEOM_HEX}[fmt or "wkb"]
        else:
            f, offsets, data, valid = geometry_column(points)
            if fmt == "hex":
                f = N.GEOM_HEX
        offsets = np.ascontiguousarray(offsets)
        if offsets.dtype == np.int32:
            f |= N.GEOM_OFFSETS32
        else:
            offsets = offsets.astype(np.int64, copy=False)
        n = len(offsets) - 1
        x, y, status = np.empty(n), np.empty(n), np.empty(n, np.uint8)
        n_rp = ctypes.c_int64(0)
        v = None if valid is None else np.ascontiguousarray(valid, dtype=np.uint8)
        N.check(N.lib().mosaic_point_geom_decode(self.handle, f, N.ptr(offsets), N.ptr(data), N.ptr(v), n, N.ptr(x),
                                                 N.ptr(y), N.ptr(status), ctypes.byref(n_rp)))
        if n_rp.value or (status == N.ROW_NULL).any():
            raise RowPathRequired(np.flatnonzero(status != N.ROW_OK))
        return x, y

    # ---- st_contains ----
    def st_contains(self, geoms, points):
        """Row-wise st_contains(geom, point): geoms are WKB bytes or WKT strings (one per row, or one
        for all rows); points as in grid_pointascellid (a point geometry column is decoded on the
        device; rows it leaves to the row path raise RowPathRequired)."""
        xy = _points_xy(points)
        if xy is None:
            xy = self.decode_points(points)
        x, y = xy
        if _is_torch(x):
            x, y = x.cpu(), y.cpu()
        x, y = np.asarray(x), np.asarray(y)
        n = len(x)
        if isinstance(geoms, (str, bytes, bytearray)):
            geoms = [geoms]
            index = np.zeros(n, np.int32)
        else:
            geoms = list(geoms)
            if len(geoms) != n:
                raise ValueError("one geometry per point row expected")
            index = np.arange(n, dtype=np.int32)
        blobs = []
        for g in geoms:
            if isinstance(g, str):
                kind, parts = W.read_wkt(g)
                if kind != "polygon":
                    raise ValueError("st_contains left side must be polygonal in this engine")
                blobs.append(W.geometry_wkb(parts) if parts else b"")
            else:
                blobs.append(bytes(g))
        lens = np.array([len(b) for b in blobs], np.int64)
        offs = np.zeros(len(blobs) + 1, np.int64)
        np.cumsum(lens, out=offs[1:])
        data = np.frombuffer(b"".join(blobs) or b"\0", dtype=np.uint8).copy()
        out = np.zeros(n, np.uint8)
        N.check(N.lib().mosaic_st_contains(self.handle, len(blobs), N.ptr(offs), N.ptr(data), N.ptr(index),
                                           N.ptr(np.ascontiguousarray(x)), N.ptr(np.ascontiguousarray(y)), n,
                                           N.ptr(out)))
        return out.astype(bool)

    # ---- the chip join ----
    def grid_tessellateexplode(self, polygons, resolution, keep_core_geom=True, densify=1):
        """grid_tessellateexplode(geom, res, keepCoreGeom) (MosaicContext.scala functions ->
        MosaicExplode.scala:70-79 -> Mosaic.getChips core/Mosaic.scala:21-87) over a PolygonSet:
        chip columns (is_core, index_id, polygon_key, wkb) with the cell classification on this
        context's GPU (mosaic_tessellate_gpu).

        H3 geometries spanning icosahedron faces are cut into per-face pieces; only a
        geometry with a vertex more than ~78 degrees from the centre of a face it meets (no gnomonic
        face plane holds it) raises MosaicError (MOSAIC_E_ARG)."""
        return tessellate(self.index_system, polygons, resolution, keep_core_geom, densify, ctx=self)

    def chip_table(self, is_core, index_id, wkb_list, polygon_key, resolution, n_polygons=None):
        """Build side: rows of grid_tessellateexplode output (MosaicExplode.scala:70-79)."""
        self.resolution_of_table = self.index_system.get_resolution(resolution)
        return ChipTable(self, is_core, index_id, wkb_list, polygon_key, n_polygons)

    def chip_table_arrays(self, chip_offsets, is_core, index_id, wkb_list, resolution):
        """Build side from grid_tessellate chip arrays, one array per polygon row (the array form of
        PointInPolygonJoin, sql/join/PointInPolygonJoin.scala:39-66); see ChipTable.from_arrays."""
        self.resolution_of_table = self.index_system.get_resolution(resolution)
        return ChipTable.from_arrays(self, chip_offsets, is_core, index_id, wkb_list)

    def pip_join_count(self, chips, x, y, out=None):
        """Quickstart join + filter + groupBy(polygon).count(): int64 count per polygon key.
        ``out`` (optional, >= n_polygons int64, host or device) receives the counts."""
        x, y = _f64(x), _f64(y)
        self._order(x, y, out)
        n = int(x.shape[0])
        if out is not None:
            counts = out
        elif _is_torch(x):
            import torch

            counts = torch.zeros(max(chips.n_polygons, 1), dtype=torch.int64, device=x.device)
        else:
            counts = np.zeros(max(chips.n_polygons, 1), np.int64)
        N.check(N.lib().mosaic_pip_join_count(self.handle, chips.handle, N.ptr(x), N.ptr(y), n, N.ptr(counts)))
        return counts[:chips.n_polygons]

    def pip_join_pairs(self, chips, x, y, capacity=None):
        """Quickstart join + filter: (row, polygon_key) pairs sorted by (row, key)."""
        x, y = _f64(x), _f64(y)
        self._order(x, y)
        n = int(x.shape[0])
        cap = capacity if capacity is not None else max(2 * n, 1024)
        while True:
            rows = np.empty(max(cap, 1), np.int64)
            keys = np.empty(max(cap, 1), np.int32)
            n_out = ctypes.c_int64(0)
            rc = N.lib().mosaic_pip_join_pairs(self.handle, chips.handle, N.ptr(x), N.ptr(y), n, N.ptr(rows),
                                               N.ptr(keys), cap, ctypes.byref(n_out))
            if rc == N.MOSAIC_E_CAPACITY:
                cap = int(n_out.value)
                continue
            N.check(rc)
            k = int(n_out.value)
            order = np.lexsort((keys[:k], rows[:k]))
            return rows[:k][order], keys[:k][order]


    def _kring(self, cells, k, loop, raw):
        strings = len(cells) and isinstance(cells[0], str)
        ids = np.array([self.index_system.parse(c) for c in cells] if strings else cells, np.int64)
        valid = None
        n = len(ids)
        if self.index_system.grid == N.GRID_H3:
            stride = max(6 * k, 1) if loop else 1 + 3 * k * (k + 1)
        else:
            stride = 8 * k if loop else 1 + 4 * k * (k + 1)
        out = np.zeros(max(n * stride, 1), np.int64)
        cnt = np.zeros(max(n, 1), np.int32)
        N.check(N.lib().mosaic_cell_kring(self.handle, self.index_system.grid, N.ptr(ids), valid, n, int(k),
                                          int(loop), N.ptr(out), N.ptr(cnt)))
        bad = np.nonzero(cnt[:n] == -2)[0]
        if len(bad):
            raise N.MosaicError(
                N.MOSAIC_E_ARG, f"grid_cellkring / grid_cellkloop: row {int(bad[0])} (cell {int(ids[bad[0]])}) is not a valid "
                "H3 cell id")
        rows = [out[i * stride:i * stride + cnt[i]] for i in range(n)]
        if raw or self.index_system.cell_id_type != "string":
            return rows
        return [[self.index_system.format(c) for c in r] for r in rows]

    def grid_cellkring(self, cells, k, raw=False):
        """grid_cellkring(cellId, k) (MosaicContext.scala:692-693 -> CellKRing.nullSafeEval ->
        IndexSystem.kRing; BNG: BNGIndexSystem.scala:216-222, the cell and its loops 1..k; H3:
        H3IndexSystem.scala:154-160, h3.kRing: hexRange order, or H3's hash-table order where the ring
        meets a pentagon)."""
        return self._kring(cells, k, False, raw)

    def grid_cellkloop(self, cells, k, raw=False):
        """grid_cellkloop(cellId, k) (MosaicContext.scala:696-697 -> CellKLoop -> IndexSystem.kLoop;
        BNG: BNGIndexSystem.scala:234-246, the valid cells at distance k; H3: H3IndexSystem.scala:
        171-177, h3.hexRing order, or the reference's kRing set-difference fallback (Scala HashSet
        order) where the ring meets a pentagon)."""
        return self._kring(cells, k, True, raw)

    def grid_cellkringexplode(self, cells, k):
        """grid_cellkringexplode (MosaicContext.scala:694-695, CellKRingExplode): one output row per
        (input row, ring cell) -- (row index array, cell array), in the reference's order."""
        return self._explode(self.grid_cellkring(cells, k, raw=True))

    def grid_cellkloopexplode(self, cells, k):
        """grid_cellkloopexplode (CellKLoopExplode): one output row per (input row, loop cell)."""
        return self._explode(self.grid_cellkloop(cells, k, raw=True))

    def _explode(self, rows):
        lens = np.array([len(r) for r in rows], np.int64)
        idx = np.repeat(np.arange(len(rows), dtype=np.int64), lens)
        cells = np.concatenate(rows) if len(rows) else np.zeros(0, np.int64)
        if self.index_system.cell_id_type == "string":
            return idx, self._serialize(cells)
        return idx, cells

    def _h3_geometry(self, cells, mode):
        ids = np.ascontiguousarray(cells, np.int64)
        n = len(ids)
        width = (2, 20, 189)[mode]
        out = np.zeros(max(n * width, 1), np.uint8 if mode == 2 else np.float64)
        cnt = np.zeros(max(n, 1), np.int32)
        N.check(N.lib().mosaic_h3_cell_geometry(self.handle, mode, N.ptr(ids), None, n, N.ptr(out), N.ptr(cnt)))
        return out, cnt[:n], width

    def grid_cellcenter(self, cells):
        """H3 h3ToGeo over a cell column (the cell centres polyfill tests, H3IndexSystem.scala:113-126):
        array [n, 2] of (lng, lat) degrees."""
        out, _, _ = self._h3_geometry(cells, 0)
        return out[:2 * len(cells)].reshape(-1, 2)

    def grid_boundary(self, cells):
        """H3IndexSystem.indexToGeometry's vertices (h3.h3ToGeoBoundary, H3IndexSystem.scala:93-100):
        per row an array [k, 2] of (lng, lat) degrees, k = 5..10 (the ring is not closed)."""
        out, cnt, w = self._h3_geometry(cells, 1)
        return [out[w * i:w * i + 2 * cnt[i]].reshape(-1, 2) for i in range(len(cells))]

    def grid_boundaryaswkb(self, cells):
        """grid_boundaryaswkb(cellId) (IndexGeometry.scala:65-75 -> IndexSystem.indexToGeometry ->
        toWKB): per row the cell polygon as JTS big-endian WKB -- BNG: the cell square (93 bytes);
        H3: the h3ToGeoBoundary ring closed with its first vertex."""
        if self.index_system.grid == N.GRID_H3:
            out, cnt, w = self._h3_geometry(cells, 2)
            return [out[w * i:w * i + cnt[i]].tobytes() for i in range(len(cells))]
        strings = len(cells) and isinstance(cells[0], str)
        ids = np.array([self.index_system.parse(c) for c in cells] if strings else cells, np.int64)
        out = np.zeros(max(93 * len(ids), 1), np.uint8)
        N.check(N.lib().mosaic_cell_boundary_wkb(self.handle, self.index_system.grid, N.ptr(ids), None, len(ids),
                                                 N.ptr(out)))
        return [out[93 * i:93 * (i + 1)].tobytes() for i in range(len(ids))]

    def grid_polyfill(self, polygons, resolution, raw=False):
        """grid_polyfill(geometry, res) (expressions/index/Polyfill.scala nullSafeEval ->
        IndexSystem.polyfill: H3IndexSystem.scala:113-126, BNGIndexSystem.scala:185-204) over a
        PolygonSet, on this context's GPU (mosaic_polyfill).  Returns one list per geometry: int64
        cells (H3), or BNG ids formatted as the reference's StringType ids unless raw=True.  A row the
        engine does not answer (an H3 search meeting a pentagon, a non-finite vertex, a BNG geometry
        without area) raises MosaicError."""
        res = self.index_system.get_resolution(resolution)
        h = ctypes.c_void_p()
        N.check(N.lib().mosaic_polyfill(self.handle, self.index_system.grid, res, len(polygons),
                                        N.ptr(polygons.geom_parts), N.ptr(polygons.part_rings),
                                        N.ptr(polygons.ring_offsets), N.ptr(polygons.xy), ctypes.byref(h)))
        try:
            n_rows, n_cells = ctypes.c_int64(0), ctypes.c_int64(0)
            N.check(N.lib().mosaic_cell_lists_info(h, ctypes.byref(n_rows), ctypes.byref(n_cells)))
            offs = np.zeros(n_rows.value + 1, np.int64)
            cells = np.zeros(max(n_cells.value, 1), np.int64)
            status = np.zeros(max(n_rows.value, 1), np.int32)
            N.check(N.lib().mosaic_cell_lists_export(h, N.ptr(offs), N.ptr(cells), N.ptr(status)))
        finally:
            N.lib().mosaic_cell_lists_destroy(h)
        bad = np.nonzero(status[:n_rows.value] != 0)[0]
        if len(bad):
            raise N.MosaicError(N.MOSAIC_E_ARG, f"grid_polyfill: rows {bad[:8].tolist()} are not supported by this "
                                                "engine (H3 search meeting a pentagon, non-finite vertex, or a "
                                                "BNG geometry without area)")
        out = [cells[offs[g]:offs[g + 1]].copy() for g in range(n_rows.value)]
        if raw or self.index_system.grid == N.GRID_H3:
            return out
        return [list(self._serialize(c)) for c in out]

    def buffer_radius(self, polygons, resolution):
        """IndexSystem.getBufferRadius(geometry, res) per geometry of a PolygonSet (the radius
        Mosaic.mosaicFill buffers by, core/Mosaic.scala:68; H3IndexSystem.scala:73-80,
        BNGIndexSystem.scala:146-149), computed on this context's GPU (H3).  float64[n]."""
        res = self.index_system.get_resolution(resolution)
        out = np.zeros(max(len(polygons), 1), np.float64)
        N.check(N.lib().mosaic_buffer_radius(self.handle, self.index_system.grid, res, len(polygons),
                                             N.ptr(polygons.geom_parts), N.ptr(polygons.part_rings),
                                             N.ptr(polygons.ring_offsets), N.ptr(polygons.xy), N.ptr(out)))
        return out[:len(polygons)]

    def st_intersects_aggregate(self, left, right):
        """left.join(right, left_index.index_id == right_index.index_id).groupBy(left_key, right_key)
        .agg(st_intersects_aggregate(left_index, right_index)) over two chip tables
        (ST_IntersectsAggregate.scala:28-39, ST_IntersectsBehaviors.scala:34-47): arrays
        (left_key int32, right_key int32, flag bool) sorted by (left_key, right_key), one row per key
        pair that shares a cell id."""
        cap = 1024
        while True:
            lk = np.empty(cap, np.int32)
            rk = np.empty(cap, np.int32)
            fl = np.empty(cap, np.uint8)
            n_out = ctypes.c_int64(0)
            rc = N.lib().mosaic_intersects_aggregate(self.handle, left.handle, right.handle, N.ptr(lk), N.ptr(rk),
                                                     N.ptr(fl), cap, ctypes.byref(n_out))
            if rc == N.MOSAIC_E_CAPACITY and n_out.value > cap:
                cap = int(n_out.value)
                continue
            N.check(rc)
            k = int(n_out.value)
            return lk[:k], rk[:k], fl[:k].astype(bool)

    def st_intersection_aggregate(self, left, right):
        """st_intersection_aggregate(left_index, right_index) grouped by (left_key, right_key) over the
        chip join (MosaicContext st_intersection_aggregate -> ST_IntersectionAggregate.scala:40-72):
        (left_key int32, right_key int32, area float64, status uint8, wkb list of bytes) sorted by key
        pair.  The WKB is the union's polygonal part as JTS writes it (big-endian; POLYGON EMPTY when
        the pieces have no area); status 1 = not answered (wkb None, area NaN): the row path."""
        h = ctypes.c_void_p()
        N.check(N.lib().mosaic_intersection_aggregate_geometry(self.handle, left.handle, right.handle, ctypes.byref(h)))
        try:
            n, nb = ctypes.c_int64(0), ctypes.c_int64(0)
            N.check(N.lib().mosaic_isect_geoms_info(h, ctypes.byref(n), ctypes.byref(nb)))
            k = int(n.value)
            lk = np.empty(k, np.int32)
            rk = np.empty(k, np.int32)
            ar = np.empty(k, np.float64)
            st = np.empty(k, np.uint8)
            off = np.empty(k + 1, np.int64)
            data = np.empty(max(int(nb.value), 1), np.uint8)
            N.check(N.lib().mosaic_isect_geoms_export(h, N.ptr(lk), N.ptr(rk), N.ptr(ar), N.ptr(st), N.ptr(off),
                                                      N.ptr(data)))
        finally:
            N.lib().mosaic_isect_geoms_destroy(h)
        wkb = [None if st[i] else bytes(data[off[i]:off[i + 1]]) for i in range(k)]
        return lk, rk, ar, st, wkb

    def st_intersection_aggregate_area(self, left, right):
        """st_area(st_intersection_aggregate(left_index, right_index)) per (left_key, right_key) group of
        the chip join (ST_IntersectionAggregate.scala; the quantity ST_IntersectionBehaviors.scala:22-135
        checks): arrays (left_key, right_key, area float64, status uint8) sorted by key pair; status 1
        marks groups the engine does not answer (a core chip without geometry, an overlay capacity
        exceeded)."""
        cap = 1 << 16  # (a call that finds more groups reports the count and is repeated once)
        while True:
            lk = np.empty(cap, np.int32)
            rk = np.empty(cap, np.int32)
            ar = np.empty(cap, np.float64)
            st = np.empty(cap, np.uint8)
            n_out = ctypes.c_int64(0)
            rc = N.lib().mosaic_intersection_aggregate(self.handle, left.handle, right.handle, N.ptr(lk), N.ptr(rk),
                                                       N.ptr(ar), N.ptr(st), cap, ctypes.byref(n_out))
            if rc == N.MOSAIC_E_CAPACITY and n_out.value > cap:
                cap = int(n_out.value)
                continue
            N.check(rc)
            k = int(n_out.value)
            return lk[:k], rk[:k], ar[:k], st[:k]


def tessellate(index_system, polygons, resolution, keep_core_geom=True, densify=1, ctx=None):
    """grid_tessellateexplode over a PolygonSet (mosaic_amd.data.PolygonSet).

    ctx=None: the host producer (mosaic_tessellate).  ctx=MosaicContext: the cell classification
    runs on the context's GPU (mosaic_tessellate_gpu), same chip set row for row.

    Returns chip columns: dict(is_core uint8, index_id int64, polygon_key int32 (geometry index),
    wkb=(offsets int64[n+1], data uint8[...])).  MosaicExplode.scala:70-79 / Mosaic.scala:21-87.
    """
    if isinstance(index_system, str):
        index_system = INDEX_SYSTEMS[index_system]()
    res = index_system.get_resolution(resolution)
    h = ctypes.c_void_p()
    if ctx is not None:
        N.check(N.lib().mosaic_tessellate_gpu(ctx.handle, index_system.grid, res, len(polygons),
                                              N.ptr(polygons.geom_parts), N.ptr(polygons.part_rings),
                                              N.ptr(polygons.ring_offsets), N.ptr(polygons.xy),
                                              int(bool(keep_core_geom)), int(densify), ctypes.byref(h)))
    else:
        N.check(N.lib().mosaic_tessellate(index_system.grid, res, len(polygons), N.ptr(polygons.geom_parts),
                                          N.ptr(polygons.part_rings), N.ptr(polygons.ring_offsets),
                                          N.ptr(polygons.xy), int(bool(keep_core_geom)), int(densify),
                                          ctypes.byref(h)))
    # zero-copy: the arrays view the chip set's own columns, which live until the last of them is
    # collected (_ChipSetOwner destroys the set)
    owner = _ChipSetOwner(h)
    n = ctypes.c_int64(0)
    nb = ctypes.c_int64(0)
    N.check(N.lib().mosaic_chip_set_info(h, ctypes.byref(n), ctypes.byref(nb)))
    n, nb = n.value, nb.value
    p = [ctypes.c_void_p() for _ in range(5)]
    N.check(N.lib().mosaic_chip_set_columns(h, *[ctypes.byref(q) for q in p]))
    is_core = owner.view(p[0], n, ctypes.c_uint8, np.uint8)
    index_id = owner.view(p[1], n, ctypes.c_int64, np.int64)
    key = owner.view(p[2], n, ctypes.c_int32, np.int32)
    offs = owner.view(p[3], n + 1, ctypes.c_int64, np.int64)
    data = owner.view(p[4], nb, ctypes.c_uint8, np.uint8) if nb else np.zeros(1, np.uint8)
    return dict(is_core=is_core, index_id=index_id, polygon_key=key, wkb=(offs, data))


def tessellate_counters():
    """(border chips clipped by the reference-style planar clip on the host, cells that fell back to
    the face-plane clip): process-wide counters of the chip producers (mosaic_tess_counters)."""
    a, b = ctypes.c_int64(0), ctypes.c_int64(0)
    N.check(N.lib().mosaic_tess_counters(ctypes.byref(a), ctypes.byref(b)))
    return a.value, b.value


class _ChipSetOwner:
    """Holds a mosaic_chip_set whose columns numpy arrays view; destroyed with the last of them."""

    def __init__(self, h):
        self.h = h

    def view(self, ptr, n, ctype, dtype):
        if n == 0 or not ptr.value:
            return np.zeros(0, dtype)
        buf = (ctype * n).from_address(ptr.value)
        buf._owner = self  # the arrays' base keeps the set alive
        return np.frombuffer(buf, dtype=dtype)

    def __del__(self):
        if self.h:
            N.lib().mosaic_chip_set_destroy(self.h)
            self.h = None
