/*
 * libmosaic_hip.so -- C ABI of the MI355X engine for Mosaic's point-in-polygon chip-join hot path.
 *
 * Plain C: pointers, sizes and status codes; no exceptions cross the boundary; no torch types.
 * Every entry point is callable from a JNI shim (the Catalyst columnar exec sketched in
 * INTEGRATION.md) or from Python ctypes (mosaic_amd/_native.py).
 *
 * Reference interfaces replaced (bransonf/mosaic @ 0.3.9, paths under
 * src/main/scala/com/databricks/labs/mosaic/):
 *   mosaic_point_to_cell      grid_pointascellid / grid_longlatascellid per row:
 *                             expressions/index/PointIndexGeom.scala:32-40,
 *                             expressions/index/PointIndexLonLat.scala:44-51 ->
 *                             core/index/H3IndexSystem.scala:140-142 (pointToIndex) and
 *                             core/index/BNGIndexSystem.scala:277-291 (pointToIndex)
 *   mosaic_point_geom_to_cell grid_pointascellid over a geometry column (WKB / WKT / hex rows):
 *   mosaic_point_geom_decode    PointIndexGeom.scala:32-40 -> GeometryAPI.geometry (GeometryAPI.scala:64-72)
 *                             -> MosaicGeometryJTS.fromWKB / fromWKT / fromHEX (MosaicGeometryJTS.scala:164,
 *                             195-200) -> getCentroid (:49-53) -> getX / getY (point/MosaicPointJTS.scala:23-25)
 *   mosaic_resolution         H3IndexSystem.getResolution (H3IndexSystem.scala:39-54),
 *                             BNGIndexSystem.getResolution (BNGIndexSystem.scala:342-353)
 *   mosaic_bng_format/_parse  BNGIndexSystem.format / parse (BNGIndexSystem.scala:114-129, 391-413)
 *   mosaic_chip_table_create  the build side of the chip join: rows of ChipType
 *                             struct<is_core, index_id, wkb> (core/types/ChipType.scala:17-28,
 *                             core/types/model/MosaicChip.scala:20-74) produced by
 *                             grid_tessellateexplode (expressions/index/MosaicExplode.scala:70-79)
 *   mosaic_pip_join_count     the Quickstart join + filter + groupBy(zone).count():
 *   mosaic_pip_join_pairs       point_cell == chip.index_id && (chip.is_core || st_contains(chip.wkb, point))
 *                             (notebooks/examples/python/QuickstartNotebook.py:205-219;
 *                             sql/join/PointInPolygonJoin.scala:68-84)
 *   mosaic_st_contains        st_contains(geom, point) per row: expressions/geometry/ST_Contains.scala:34-42
 *                             -> core/geometry/MosaicGeometryJTS.scala:101 (JTS Geometry.contains)
 *
 * Conventions
 *   - Return value: MOSAIC_OK (0) or a mosaic_status code; mosaic_last_error() (thread-local)
 *     holds the message.  MOSAIC_E_RES / MOSAIC_E_NAN carry the reference's exception messages
 *     ("H3 resolution has to be between 0 and 15; found N", "BNG resolution not supported; found N",
 *     "NaN coordinates are not supported.") so a JNI shim can rethrow IllegalStateException.
 *   - Input arrays are borrowed for the duration of the call and may live in host memory or in
 *     device memory of the context's GPU (detected per pointer).  Host inputs are staged over PCIe.
 *     Device inputs must be complete when the call's work starts: the context's own streams are
 *     non-blocking (no implicit order with the null stream), so a caller producing columns on another
 *     stream binds that stream with mosaic_set_stream, records an event on it and passes it to
 *     mosaic_stream_wait_event before the call, or synchronises it first.
 *   - Calls are synchronous unless the context option "async" is 1, in which case device-pointer
 *     calls only enqueue work on the calling thread's stream (mosaic_sync() waits and reports
 *     deferred errors).  Exception: a binned join (option "bin_points", tables without a usable point
 *     raster) reads its kept-row count back once per sort chunk, so it blocks the calling thread
 *     until each chunk's cover pass has run; its results are still reported through mosaic_sync.
 *   - Threads: a context is bound to one GPU and every entry point is thread-safe (SURVEY.md §8(b),
 *     the executor's task threads sharing one context; the reference's index systems are JVM
 *     singletons, H3IndexSystem.scala:22-27).  Each calling thread gets its own HIP stream (created
 *     on first use; mosaic_set_stream / mosaic_get_stream act on the calling thread's), scratch
 *     buffers, counters (mosaic_last_stats) and timing events, so concurrent calls never share
 *     state.  Options are shared by the context and copied once at the start of every call.  Chip
 *     tables are immutable once created and may be joined from any thread.
 */
#ifndef MOSAIC_HIP_H
#define MOSAIC_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: mosaic_chip_table_raster writes 8 values (was 5); option "exact_cap"; the aggregate geometry.
 * 3: mosaic_chip_table_raster writes 9 values (out9[8] = leaf_lines; callers must pass 9 slots);
 *    mosaic_intersection_aggregate_geometry; mosaic_cell_kring count -4 for rows with k > 128 near a
 *    pentagon (now answered, see 4).
 * 4: border chips are the reference's planar clip against indexToGeometry (mosaic_tessellate);
 *    mosaic_tess_counters; mosaic_cell_kring answers every row (no -4). */
#define MOSAIC_ABI_VERSION 4

typedef enum {
    MOSAIC_OK = 0,
    MOSAIC_E_ARG = 1,      /* invalid argument (null pointer, bad size, bad option) */
    MOSAIC_E_RES = 2,      /* unsupported resolution (IllegalStateException in the reference) */
    MOSAIC_E_NAN = 3,      /* NaN coordinate with BNG (IllegalStateException in the reference) */
    MOSAIC_E_HIP = 4,      /* HIP runtime error / no device */
    MOSAIC_E_WKB = 5,      /* undecodable or unsupported chip WKB */
    MOSAIC_E_CAPACITY = 6, /* output buffer too small (pairs) or deferred queue overflow (async) */
    MOSAIC_E_NOMEM = 7     /* allocation failure */
} mosaic_status;

typedef enum { MOSAIC_GRID_H3 = 0, MOSAIC_GRID_BNG = 1 } mosaic_grid;

typedef struct mosaic_ctx mosaic_ctx;
typedef struct mosaic_chips mosaic_chips;

int mosaic_abi_version(void);
const char* mosaic_last_error(void);

/* ---- context ---- */
/* Bind a context to HIP device `device` (ordinal as seen by this process). */
int mosaic_init(int device, mosaic_ctx** out);
int mosaic_destroy(mosaic_ctx* ctx);
/* Options: "jdk" (8: Math.toRadians = deg / 180 * PI, the JDK 8 runtime of the reference's CI;
 * 9+: deg * DEGREES_TO_RADIANS), "async" (0/1), "block" (threads per block of the row kernels,
 * multiple of 64), "blocks_per_cu" (grid sizing), "timing" (0/1: HIP events around each join's main
 * kernel; 2: the point-raster join's mixed-cell kernel is timed as a second entry), "raster" (ray-parity
 * raster cells per border chip side, 1..64, for tables built afterwards), "raster_adaptive" (0/1: rings
 * with few segments get 2 ceil(sqrt(segments)) cells a side instead, at most "raster"; default 1),
 * "raster_min_segments" (rings with fewer segments get no raster: their contains test walks the
 * segments; default 0, and at least 16 for H3 tables with more polygons than point-raster codes,
 * whose joins test chips from tile images instead),
 * "lane_edges" (raster cell lists up to this long are evaluated by the owning lane), "tiles" (0/1: H3
 * tile directory for tables built afterwards, and its use by joins), "point_raster" (0/1: the point
 * raster over the tile directory, likewise), "raster_sub" / "raster_cell" (its sub-blocks per tile
 * side and leaf cells per sub-block side, powers of two, for tables built afterwards; default 64 /
 * 16), "raster_lines" (0/1: sub-blocks crossed by one straight chip edge store a line record instead
 * of a leaf block; default 1), "raster_leaf_lines" (0/1: leaf cells of the other mixed sub-blocks
 * crossed by one straight chip edge store a line record too, answered by k_join_leaf before
 * k_join_mixed; default 1 since round 6: the reference's chord-edged border chips leave ~1.6x more
 * mixed leaf rows than face-plane chips did), "leaf_join" (0/1: joins run k_join_leaf on the mixed queue; default 1),
 * "raster_build" (1: the point raster is classified on the GPU, the
 * default; 0: on host threads -- identical bytes), "raster_quad" (its LDS level: 0 off, 1 default budget of 32768
 * entries, or an entry budget <= 65536), "stream_block" (k_join_stream workgroup size, a multiple of
 * 64 up to 1024, default 1024), "host_chunk" (rows per chunk when mosaic_pip_join_count gets
 * host-resident coordinates: the next chunk's copy overlaps the current chunk's join; 0 = stage the
 * whole batch; default 2^25), "mixed_rows" (1/2/4, default 1), "mixed_blocks_per_cu" (default 16), "cell_blocks_per_cu" (k_cell_h3 grid, default 256; 0 = one lane per row pair), "stream_pipe"
 * (0: k_join_stream; 1: the software-pipelined H3 stream kernel; 2: it with the gathering rows
 * compacted, k_join_stream_cpt, the default -- each where it applies), "bng_cpt" (0/1: the compacted
 * BNG stream kernel where it applies; default 1), "bng_lds" (0/1: BNG tables
 * built afterwards carry an LDS cell level for the BNG stream kernel; default 1), "bng_cell" (sub-cells
 * per BNG border cell side in those tables, a power of two <= 64; default 32), "bng_group_lines" (0/1:
 * those tables' sub-block levels name a line record wherever one decides a whole 4 x 4 group; default
 * 1), "bng_wedges" (0/1: those tables carry wedge records for sub-cells split at a chip vertex,
 * answered by the BNG mixed-row kernel before its chip loop; default 1), "scratch_limit" (see
 * the per-thread state below), "bin_points" (0/1: H3 joins on a tile directory without a usable point
 * raster sort the points by tile before the chip loop -- the border-chip-heavy C4 shape; default 1),
 * "bin_min_rows" (smallest batch that is binned; default 2^18), "bin_chunk" (rows per sort chunk;
 * default 2^28), "tile_images" (0: none; 1: tables built without a point raster carry per-tile chip
 * images the binned join copies into LDS, the default; 2: every tile-directory table carries them),
 * "bin_spin_cap" (the binned join's look-back poll limit; < 0 forces its uncompacted fallback -- a test
 * knob), "exact_cap" (rows of the exact-H3 queue; 0 = the default max(n / 8, 2^20) capped at n; an overflow
 * reruns the batch on the exact path, or is reported as MOSAIC_E_CAPACITY by mosaic_sync after an
 * async call). */
int mosaic_set_option(mosaic_ctx* ctx, const char* key, int64_t value);
/* Per-thread state.  Each calling thread gets its own execution state on a context (HIP stream,
 * copy stream, timing events, scratch queues and staging sized by its largest call).  It is freed
 * by mosaic_thread_release (the calling thread's state), by mosaic_destroy (all), or when a thread
 * other than the process's main thread exits (a thread_local guard), so an executor whose worker
 * pool retires and creates threads does not accumulate streams or scratch.  States are keyed by a
 * per-thread serial number, never by pthread ids (which the runtime reuses).  Option
 * "scratch_limit" (bytes, 0 = keep; default 0) frees a thread's scratch when a call returns holding
 * more than that.  mosaic_thread_count reports the live states and the scratch they hold.
 * (Replaces no reference interface: the JVM side's H3Core / index-system singletons hold no device
 * state, H3IndexSystem.scala:22-27; this is the multiplexing SURVEY.md §8(b) asks of the ABI.) */
int mosaic_thread_release(mosaic_ctx* ctx);
int mosaic_thread_count(mosaic_ctx* ctx, int64_t* n_threads, int64_t* scratch_bytes);
/* The calling thread's hipStream_t (created by the context unless set by this thread). */
int mosaic_get_stream(mosaic_ctx* ctx, void** stream);
int mosaic_set_stream(mosaic_ctx* ctx, void* stream);
/* Orders the calling thread's later work after a caller event: enqueues hipStreamWaitEvent(stream,
 * (hipEvent_t)event) on the thread's stream, so device columns produced on another stream (a cuDF /
 * Arrow producer, torch) are complete before the next call reads them, without binding that stream
 * or blocking the host.  The event must have been recorded (hipEventRecord) before this call. */
int mosaic_stream_wait_event(mosaic_ctx* ctx, void* event);
/* Wait for enqueued work; reports deferred errors of async calls. */
int mosaic_sync(mosaic_ctx* ctx);
/* Counters of the calling thread's last join/index call: [0] rows that needed the exact H3 path,
 * [1] (point, border chip) contains tests, [2] matched pairs (pairs calls only).
 * Filled only by sync calls. */
int mosaic_last_stats(mosaic_ctx* ctx, int64_t* out3);
/* Rows the calling thread's last join sorted on its binned path (the points some chip may hold:
 * k_bin_cover's keep count), 0 when the join took another path. */
int mosaic_last_binned_rows(mosaic_ctx* ctx, int64_t* out);
/* With option "timing" = 1, every join call brackets its fused kernel with HIP events on the
 * context stream.  Waits for the stream, writes up to cap elapsed times (ms) in call order, reports
 * how many calls were timed in *n_out, and resets the list. */
int mosaic_kernel_times(mosaic_ctx* ctx, double* out_ms, int64_t cap, int64_t* n_out);
/* Name of the dominant kernel of the calling thread's last join call ("k_join_stream_cpt",
 * "k_join_stream_pipe", "k_join_stream_bng", ...; "" before any): what a profile of that call
 * should be filtered on.  Static storage; never freed. */
const char* mosaic_last_kernel(mosaic_ctx* ctx);

/* ---- grid systems ---- */
/* getResolution for an Int resolution; validates the range of the grid system. */
int mosaic_resolution(int grid, int res, int* out);
/* getResolution for a String resolution ("9" for H3; "100m", "500m", ... or "4" for BNG). */
int mosaic_resolution_str(int grid, const char* res, int* out);
/* grid_pointascellid / grid_longlatascellid: x = lon (H3) or easting (BNG), y = lat or northing.
 * valid (nullable): 1 = row present; null rows give out_valid 0 and cell 0 (NullIntolerant). */
int mosaic_point_to_cell(mosaic_ctx* ctx, int grid, int res, const double* x, const double* y,
                         const uint8_t* valid, int64_t n, int64_t* out_cell, uint8_t* out_valid);
/* H3 cells from the exact path alone (h3_exact: the line-by-line H3 C v3.7 restatement with the
 * glibc 2.35 libm restatement glibc_math.h) for every row, skipping the certified fast path;
 * x = lon, y = lat (degrees).  Same answer as mosaic_point_to_cell; exists so the exact path can be
 * checked against the reference on arbitrarily many rows. */
int mosaic_point_to_cell_exact(mosaic_ctx* ctx, int res, const double* x, const double* y, int64_t n,
                               int64_t* out_cell);
/* Diagnostics: out[i] = the device's glibc restatement of fn(a[i]) / atan2(a[i], b[i]);
 * fn 0 = sin, 1 = cos (both via sincos), 2 = tan, 3 = acos, 4 = atan2. */
int mosaic_diag_libm(mosaic_ctx* ctx, int fn, const double* a, const double* b, int64_t n, double* out);
/* grid_pointascellid over a point geometry column in Arrow binary / utf8 layout: row i is
 * data[offsets[i] .. offsets[i+1]); format = MOSAIC_GEOM_WKB / _WKT / _HEX, | MOSAIC_GEOM_OFFSETS32
 * for 32-bit offsets (default 64-bit).  Every row JTS 1.19 certainly reads as a non-empty Point is
 * decoded on the device (Double.parseDouble-exact numbers; either WKB byte order; EWKB / ISO Z, M,
 * SRID) and indexed: row_status MOSAIC_ROW_OK.  Null rows: MOSAIC_ROW_NULL, cell 0.  Every other
 * row (other geometry types, whose centroid the reference indexes; POINT EMPTY and malformed rows,
 * on which the reference throws) gets MOSAIC_ROW_PATH and cell 0: the caller evaluates those rows
 * with the reference's row-wise expression.  *n_rowpath (nullable) = their number. */
#define MOSAIC_GEOM_WKB 0
#define MOSAIC_GEOM_WKT 1
#define MOSAIC_GEOM_HEX 2
#define MOSAIC_GEOM_OFFSETS32 0x100
#define MOSAIC_ROW_NULL 0
#define MOSAIC_ROW_OK 1
#define MOSAIC_ROW_PATH 2
int mosaic_point_geom_to_cell(mosaic_ctx* ctx, int grid, int res, int format, const void* offsets,
                              const uint8_t* data, const uint8_t* valid, int64_t n, int64_t* out_cell,
                              uint8_t* row_status, int64_t* n_rowpath);
/* The decode alone: x / y of MOSAIC_ROW_OK rows (0 elsewhere), row_status as above. */
int mosaic_point_geom_decode(mosaic_ctx* ctx, int format, const void* offsets, const uint8_t* data,
                             const uint8_t* valid, int64_t n, double* x, double* y, uint8_t* row_status,
                             int64_t* n_rowpath);
/* grid_pointascellid over the COORDS form of points: InternalGeometryType rows
 * struct<typeId: int, srid: int, boundaries: array<array<array<double>>>, holes: ...>
 * (core/types/model/InternalGeometry.scala; st_point's output, expressions/constructors/ST_Point.scala:27-32)
 * as Arrow columns: type_id[n]; boundary_offsets[n + 1] (row -> boundaries), coord_offsets
 * (boundary -> coordinates), value_offsets (coordinate -> values), all int32 (Arrow list); values
 * (float64).  Rows with type_id 1 (POINT) whose first boundary's first coordinate has 2 values, or
 * 3 or more (z ignored), are decoded as MosaicPointJTS.fromInternal does
 * (core/geometry/point/MosaicPointJTS.scala:82-89) and indexed: MOSAIC_ROW_OK.  Null rows:
 * MOSAIC_ROW_NULL.  Other types (the reference indexes their centroid) and rows the reference throws
 * on (no boundary, no coordinate, a 1-value coordinate): MOSAIC_ROW_PATH.  Child arrays must not
 * hold nulls.  The holes column is not read (a Point has none). */
int mosaic_point_coords_to_cell(mosaic_ctx* ctx, int grid, int res, const int32_t* type_id,
                                const int32_t* boundary_offsets, const int32_t* coord_offsets,
                                const int32_t* value_offsets, const double* values, const uint8_t* valid, int64_t n,
                                int64_t* out_cell, uint8_t* row_status, int64_t* n_rowpath);
/* The decode alone: x / y of MOSAIC_ROW_OK rows (0 elsewhere), row_status as above. */
int mosaic_point_coords_decode(mosaic_ctx* ctx, const int32_t* type_id, const int32_t* boundary_offsets,
                               const int32_t* coord_offsets, const int32_t* value_offsets, const double* values,
                               const uint8_t* valid, int64_t n, double* x, double* y, uint8_t* row_status,
                               int64_t* n_rowpath);
/* BNG id <-> string (BNGIndexSystem.format / parse).  format returns the string length. */
int mosaic_bng_format(int64_t id, char* buf, size_t cap);
int mosaic_bng_parse(const char* s, int64_t* out);
/* serializeCellId over a BNG cell column (IndexSystem.scala:37-46 -> BNGIndexSystem.format
 * :114-129), computed on the GPU, in Arrow utf8 layout: offsets[n + 1] (int64) and the characters.
 * Null rows (valid[i] == 0; valid may be null) are empty strings.  If the characters exceed
 * chars_cap, returns MOSAIC_E_CAPACITY with *chars_needed set (offsets are written either way);
 * an id the reference cannot format gives MOSAIC_E_ARG. */
int mosaic_bng_format_column(mosaic_ctx* ctx, const int64_t* ids, const uint8_t* valid, int64_t n, int64_t* offsets,
                             char* chars, int64_t chars_cap, int64_t* chars_needed);

/* BNGIndexSystem.parse (BNGIndexSystem.scala:391-413) over a string column on the GPU: the
 * StringType cell ids of BNG chips (BNGIndexSystem.scala:28, serializeCellId IndexSystem.scala:37-46)
 * back to the long ids mosaic_chip_table_create takes.  Arrow utf8 (offsets32 = 1: int32 offsets) or
 * large_utf8 (int64 offsets) layout, offsets[n + 1] + chars; null rows (valid[i] == 0) give 0.
 * A row the reference cannot parse (its letterMap lookup or Integer.parseInt throws) gives
 * MOSAIC_E_ARG naming the first such row. */
int mosaic_bng_parse_column(mosaic_ctx* ctx, int offsets32, const void* offsets, const uint8_t* chars,
                            const uint8_t* valid, int64_t n, int64_t* out_ids);

/* ---- chip table (build side) ---- */
/* n_chips rows of ChipType: is_core[i], index_id[i] (int64 cell id), wkb bytes
 * wkb[wkb_offsets[i] .. wkb_offsets[i+1]) (Polygon / MultiPolygon, either byte order; empty or
 * zero-length = no geometry), polygon_key[i] in [0, n_polygons) (the row's zone / group key).
 * The table is copied to device memory; the caller may free its buffers after the call. */
int mosaic_chip_table_create(mosaic_ctx* ctx, int grid, int res, int64_t n_chips, const uint8_t* is_core,
                             const int64_t* index_id, const int64_t* wkb_offsets, const uint8_t* wkb,
                             const int32_t* polygon_key, int32_t n_polygons, mosaic_chips** out);
/* The same over Arrow columns as a JNI shim hands them over: wkb_offsets are int32 (Arrow binary)
 * when wkb_offsets32 != 0, else int64 (large_binary).  BNG StringType ids: parse them first with
 * mosaic_bng_parse_column. */
int mosaic_chip_table_create_arrow(mosaic_ctx* ctx, int grid, int res, int64_t n_chips, const uint8_t* is_core,
                                   const int64_t* index_id, const void* wkb_offsets, int wkb_offsets32,
                                   const uint8_t* wkb, const int32_t* polygon_key, int32_t n_polygons,
                                   mosaic_chips** out);
/* The array form (PointInPolygonJoin.joinArrayRows, sql/join/PointInPolygonJoin.scala:39-66): polygon
 * row p's chip array (grid_tessellate's chips) is rows [chip_offsets[p], chip_offsets[p + 1]) of the
 * flattened columns is_core / index_id / wkb (wkb_offsets indexed from chip_offsets[0], n + 1 entries);
 * joins then count at most one pair per (point, polygon row), from the first chip of the row with
 * the point's cell (array_position + element_at), as the reference does. */
int mosaic_chip_table_create_arrays(mosaic_ctx* ctx, int grid, int res, int32_t n_polygons, const int64_t* chip_offsets,
                                    const uint8_t* is_core, const int64_t* index_id, const int64_t* wkb_offsets,
                                    const uint8_t* wkb, mosaic_chips** out);
int mosaic_chip_table_destroy(mosaic_chips* chips);
/* out8: n_chips, n_cells, n_border, n_vertices, n_rings, device_bytes, hash_capacity, n_polygons */
int mosaic_chip_table_info(const mosaic_chips* chips, int64_t* out8);

/* H3 tile directory of the table (built when option "tiles" = 1, the default): out13 = built (0/1),
 * tiles along lon, tiles along lat, tile records, window entries, tiles on the generic path, rings;
 * point raster (option "point_raster" = 1, the default) built (0/1), sub-blocks per tile side,
 * cells per sub-block side, pure sub-blocks, mixed sub-blocks, mixed cells.  BNG tables report their
 * dense cell table instead in the first five: built (0/1), cells along e, cells along n, bytes of the
 * LDS cell level (option "bng_lds"), its block shift, mixed border-cell sub-cells, line-record sub-cells. */
int mosaic_chip_table_tiles(const mosaic_chips* chips, int64_t* out13);
/* out4 = lon, lat of the tile grid origin and tiles per degree along lon, lat (tile i covers
 * [x0 + i / sx, x0 + (i + 1) / sx)). */
int mosaic_chip_table_tile_grid(const mosaic_chips* chips, double* out4);
/* Point raster detail: out5 = sub-blocks stored as line records (option "raster_lines"), LDS quad
 * level entries (0: none), quad shift (sub-blocks per quad side = 1 << shift), raster bytes on the
 * device, 1 if joins run the stream kernel on it (quad level with compact copies, edges clamp-safe);
 * then the binned join's per-tile LDS chip images (option "tile_images"): records with an image,
 * image bytes on the device, bytes of the largest image; leaf cells stored as line records (option
 * "raster_leaf_lines"). */
int mosaic_chip_table_raster(const mosaic_chips* chips, int64_t* out9);
/* Build cost of the table in ms (ms4): chip hash + geometry + chip rasters, tile directory (host),
 * point-raster classification (GPU with option "raster_build" = 1, the default; host threads with
 * 0), point-raster assembly (host); *digest = FNV-1a 64 of the point raster's arrays (0: no raster),
 * equal for both classification builds. */
int mosaic_chip_table_build_info(const mosaic_chips* chips, double* ms4, uint64_t* digest);

/* ---- the join ---- */
/* counts[p] = number of (point, chip) pairs with chip polygon_key p (overwritten). */
int mosaic_pip_join_count(mosaic_ctx* ctx, const mosaic_chips* chips, const double* x, const double* y,
                          int64_t n, int64_t* counts);
/* Emits every matching (row, polygon_key) pair (unordered).  If more than `cap` pairs match,
 * returns MOSAIC_E_CAPACITY with *n_out = required size. */
int mosaic_pip_join_pairs(mosaic_ctx* ctx, const mosaic_chips* chips, const double* x, const double* y,
                          int64_t n, int64_t* out_row, int32_t* out_key, int64_t cap, int64_t* n_out);

/* ---- chip production (host; build side of the join, not the hot path) ---- */
/* grid_tessellateexplode(geometry, res, keep_core_geom) over n_geoms polygonal geometries given as
 * flat rings: geometry g = parts [geom_parts[g], geom_parts[g+1]); part p = rings
 * [part_rings[p], part_rings[p+1]); ring r = vertices xy[2*ring_offsets[r] ..] (x, y interleaved,
 * lon/lat for H3, BNG metres for BNG).  Chip rows carry the geometry index as their key.
 * Cells are enumerated and classified (core / border / none) in the plane where they are exact
 * (H3: the icosahedron face's gnomonic plane; BNG: metres).  A border chip is the reference's
 * `geometry.intersection(indexToGeometry(cell))` (IndexSystem.getBorderChips): the geometry clipped
 * in its own coordinates against the cell polygon -- H3: the h3ToGeoBoundary ring in degrees (JDK 8
 * Math.toDegrees) with straight sides, face-edge vertices included; BNG: the square -- with JTS
 * 1.19's crossing arithmetic (RobustLineIntersector / Intersection.intersection), every ring written
 * from its lowest vertex, shells counter-clockwise, holes clockwise, polygons by lowest vertex (the
 * order of the reference's rendered chips); a border chip equal to its cell is a core chip
 * (`intersect.equals(indexGeom)`).  A core chip's geometry is indexToGeometry(cell) (densify > 1: H3
 * core outlines follow the cell's arcs with `densify` points a side instead).  Cells the planar clip
 * cannot take (over the antimeridian or a pole) are clipped in the face plane instead
 * (mosaic_tess_counters counts them).  MOSAIC_E_ARG for a geometry with a vertex more than ~78 degrees
 * from the centre of a face it meets.
 * Reference: expressions/index/MosaicExplode.scala:70-79, core/Mosaic.scala:21-87,
 * core/index/IndexSystem.scala:152-186, core/index/H3IndexSystem.scala:93-100. */
typedef struct mosaic_chip_set mosaic_chip_set;
int mosaic_tessellate(int grid, int res, int64_t n_geoms, const int64_t* geom_parts, const int64_t* part_rings,
                      const int64_t* ring_offsets, const double* xy, int keep_core_geom, int densify,
                      mosaic_chip_set** out);
int mosaic_chip_set_info(const mosaic_chip_set* cs, int64_t* n_chips, int64_t* wkb_bytes);
/* Copies the chip rows out: is_core[n], index_id[n], key[n], wkb_offsets[n+1], wkb[wkb_bytes]. */
/* Zero-copy view of the same columns: pointers into the chip set, valid until mosaic_chip_set_destroy
 * (what mosaic_chip_set_export copies; the Python binding wraps them and destroys the set with the
 * last array). */
int mosaic_chip_set_columns(const mosaic_chip_set* cs, const uint8_t** is_core, const int64_t** index_id,
                            const int32_t** key, const int64_t** wkb_offsets, const uint8_t** wkb);
int mosaic_chip_set_export(const mosaic_chip_set* cs, uint8_t* is_core, int64_t* index_id, int32_t* key,
                           int64_t* wkb_offsets, uint8_t* wkb);
int mosaic_chip_set_destroy(mosaic_chip_set* cs);
/* grid_tessellateexplode with the cell classification on the GPU: the same chip set as
 * mosaic_tessellate, row for row and byte for byte.  Each candidate cell of a geometry's envelope is
 * classified on the GPU (border: a ring segment within eps of the cell; core: cell centre inside
 * the part, even-odd; else dropped), replacing the per-cell JTS buffer / intersects of
 * IndexSystem.getBorderChips / getCoreChips (core/index/IndexSystem.scala:152-186, via
 * Mosaic.mosaicFill core/Mosaic.scala:60-87).  BNG: k_bng_tess_classify on the cell squares; H3:
 * k_tess_classify_poly on the (densify-subdivided) hexagons in the icosahedron face plane.  Border
 * cells are clipped on the GPU as well (k_tess_clip_ll, one lane per cell, the host routine's
 * arithmetic); candidate enumeration, the per-face pieces of H3 geometries spanning faces and the
 * chip WKB assembly are host code.  Errors as mosaic_tessellate. */
int mosaic_tessellate_gpu(mosaic_ctx* ctx, int grid, int res, int64_t n_geoms, const int64_t* geom_parts,
                          const int64_t* part_rings, const int64_t* ring_offsets, const double* xy,
                          int keep_core_geom, int densify, mosaic_chip_set** out);
/* Duration (HIP events on the context stream) of the last classification launch, ms. */
double mosaic_tess_last_classify_ms(const mosaic_ctx* ctx);
/* Process-wide counters of the chip producers' host clip: border chips clipped (ll_chips) and cells
 * that fell back to the face-plane clip (ll_fallbacks). */
int mosaic_tess_counters(int64_t* ll_chips, int64_t* ll_fallbacks);

/* ---- st_contains per row ---- */
/* out[i] = JTS contains(geometry[geom_index[i]], POINT(px[i] py[i])); geometries given as WKB. */
int mosaic_st_contains(mosaic_ctx* ctx, int64_t n_geoms, const int64_t* wkb_offsets, const uint8_t* wkb,
                       const int32_t* geom_index, const double* px, const double* py, int64_t n, uint8_t* out);

/* ---- st_intersects_aggregate over the chip join of two chip tables ---- */
/* For every (left polygon_key, right polygon_key) pair whose chip sets share at least one cell id,
 * flag = OR over the chip pairs of the shared cells of (left.is_core || right.is_core ||
 * JTS 1.19 intersects(left.wkb, right.wkb)).  Groups are written sorted by (left key, right key);
 * if more than `cap` groups exist, returns MOSAIC_E_CAPACITY with *n_out = the required size.
 * Both tables must use the same grid and resolution.  Replaces the equi-join + groupBy +
 * st_intersects_aggregate pattern: ST_IntersectsAggregate.update
 * (expressions/geometry/ST_IntersectsAggregate.scala:28-39) as used in
 * ST_IntersectsBehaviors.scala:34-47 / MosaicContext.scala st_intersects_aggregate. */
int mosaic_intersects_aggregate(mosaic_ctx* ctx, const mosaic_chips* left, const mosaic_chips* right,
                                int32_t* out_left_key, int32_t* out_right_key, uint8_t* out_flag, int64_t cap,
                                int64_t* n_out);

/* ---- st_intersection_aggregate over the chip join of two chip tables ---- */
/* For every (left polygon_key, right polygon_key) pair whose chip sets share a cell id: the union
 * ST_IntersectionAggregate.update / merge (expressions/geometry/ST_IntersectionAggregate.scala:40-72)
 * builds from, per joined chip pair, the cell (both core: indexToGeometry), the other chip (one core)
 * or the two chips' intersection.  Per cell that union is (the group's left chips there, or the
 * cell when one is core) n (its right chips, likewise); a cell with one pair is the pair's piece.
 * mosaic_intersection_aggregate returns its area per group -- st_area(st_intersection_aggregate(..)),
 * the quantity the reference's tests check (ST_IntersectionBehaviors.scala:22-135, 1e-8): per cell the
 * area of that piece from the cell overlay (overlay.h, one GPU lane per (group, cell)).  out_status 1
 * marks groups the engine does not answer (an overlay capacity exceeded, a cell without geometry):
 * evaluate those on the row path.  Sorted by key pair;
 * MOSAIC_E_CAPACITY with *n_out set when more than cap groups exist.  Each (group, cell) piece is one
 * record and a group's area is summed on the host in cell-slot order, so repeated calls return the
 * same bits. */
int mosaic_intersection_aggregate(mosaic_ctx* ctx, const mosaic_chips* left, const mosaic_chips* right,
                                  int32_t* out_left_key, int32_t* out_right_key, double* out_area, uint8_t* out_status,
                                  int64_t cap, int64_t* n_out);
/* The aggregate's geometry: per group the union as the WKB JTS writes (big-endian 2D Polygon, or
 * MultiPolygon for several polygons; POLYGON EMPTY when the pieces have no area), dissolved across
 * cells (pieces of adjacent cells form one polygon; shells clockwise, holes counter-clockwise).  The
 * per-cell boundaries come from the GPU (overlay.h, one lane per (group, cell)); the host joins them
 * (isect_geom.cpp).  Lower-dimensional parts of the reference's result (chips that only touch, whose
 * JTS intersection is a line or a point) are not emitted: the polygonal part is.  Vertex order and
 * ring starts are not JTS's (the reference's own depend on Spark's aggregation order).  area = the
 * sum of the cells' piece areas (cell-slot order); status 1 = not answered (area NaN, no WKB). */
typedef struct mosaic_isect_geoms mosaic_isect_geoms;
int mosaic_intersection_aggregate_geometry(mosaic_ctx* ctx, const mosaic_chips* left, const mosaic_chips* right,
                                           mosaic_isect_geoms** out);
int mosaic_isect_geoms_info(const mosaic_isect_geoms* g, int64_t* n_groups, int64_t* wkb_bytes);
/* left_key[n], right_key[n], area[n], status[n], wkb_offsets[n + 1], wkb[wkb_bytes] (any may be null) */
int mosaic_isect_geoms_export(const mosaic_isect_geoms* g, int32_t* left_key, int32_t* right_key, double* area,
                              uint8_t* status, int64_t* wkb_offsets, uint8_t* wkb);
int mosaic_isect_geoms_destroy(mosaic_isect_geoms* g);

/* ---- grid_cellkring / grid_cellkloop over a cell column (BNG, H3) ---- */
/* loop = 0: kRing(cell, k); loop = 1: kLoop(cell, k).  Row i's cells go to out[i * stride ..] and
 * out_count[i] = their number (-1 for null rows, valid[i] == 0).  0 <= k <= 1000.
 * BNG: stride = 8k (loop) or 1 + 4k(k + 1) (ring), the cell then the loops 1..k, in the reference's
 * order (bottom, right, top, left; cells failing isValid dropped).  Reference: BNGIndexSystem.kRing /
 * kLoop / isValid (core/index/BNGIndexSystem.scala:216-263).
 * H3: stride = max(6k, 1) (loop) or 1 + 3k(k + 1) (ring), in H3 v3.7's hexRange / hexRing order
 * (reference H3IndexSystem.kRing / kLoop, core/index/H3IndexSystem.scala:154-177); where the walk
 * meets a pentagon, kRing is H3's _kRingInternal hash table read in slot order (as h3-java returns
 * it) and kLoop the reference's own fallback, kRing(k).toSet diff kRing(k - 1).toSet in Scala
 * HashSet order (:169-176).  That search makes ~5 k^3 dependent steps per row: it runs on the GPU for
 * k <= 128 and on host threads beyond (the same code), so every row is answered.  A row whose id is
 * not a valid cell gets out_count[i] = -2 (no cells written). */
int mosaic_cell_kring(mosaic_ctx* ctx, int grid, const int64_t* cells, const uint8_t* valid, int64_t n, int k,
                      int loop, int64_t* out, int32_t* out_count);

/* ---- H3 cell geometry over a cell column ---- */
/* H3 C v3.7 h3ToGeo / h3ToGeoBoundary bit for bit (x87 long-double steps and glibc libm restated),
 * in degrees through java.lang.Math.toDegrees (option "jdk"), x = lng, y = lat.
 * mode 0 (h3ToGeo): out = double[2 n], the cell centre (x, y); out_count[i] = 1.
 * mode 1 (h3ToGeoBoundary): out = double[20 n], row i's vertices from out + 20 i as (x, y) pairs;
 *   out_count[i] = their number (5..10: Class III cells crossing an icosahedron edge and pentagons
 *   carry extra edge vertices).
 * mode 2 (grid_boundaryaswkb: IndexGeometry -> H3IndexSystem.indexToGeometry -> toWKB): out =
 *   uint8[189 n], row i's JTS big-endian 2D WKB polygon (the boundary closed with its first vertex)
 *   from out + 189 i; out_count[i] = its byte length (13 + 16 (vertices + 1)).
 * Null rows (valid[i] == 0): out_count[i] = -1.  An id that is not a valid H3 cell: MOSAIC_E_ARG.
 * Reference: H3IndexSystem.indexToGeometry / getBufferRadius / polyfill
 * (core/index/H3IndexSystem.scala:73-126), expressions/index/IndexGeometry.scala:65-75. */
int mosaic_h3_cell_geometry(mosaic_ctx* ctx, int mode, const int64_t* cells, const uint8_t* valid, int64_t n,
                            void* out, int32_t* out_count);

/* ---- grid_polyfill ---- */
/* grid_polyfill(geometry, res) over n_geoms polygonal geometries in the flat-ring layout of
 * mosaic_tessellate (x = lon, y = lat for H3; BNG metres), on the GPU.  Row g's cells are
 * cells[offsets[g] .. offsets[g + 1]) of the result (mosaic_cell_lists_export).
 * H3: per polygon part, H3 C v3.7 polyfill(shell, holes, res) as h3-java 3.7.0 is called by
 * H3IndexSystem.polyfill (core/index/H3IndexSystem.scala:113-126): the cells whose h3ToGeo centre
 * H3's pointInsidePolygon accepts, reached from the cells of the sampled ring edges; the parts' lists
 * concatenated, each in the order h3-java returns (H3's output-table slot order).  Vertices through
 * Math.toRadians (option "jdk").
 * BNG: BNGIndexSystem.polyfill (core/index/BNGIndexSystem.scala:185-204): the cells reached from
 * the vertex and centroid cells whose square's centroid the geometry contains (JTS), ordered as
 * the reference's Scala immutable HashSet iterates them.
 * status[g]: MOSAIC_POLYFILL_OK, or MOSAIC_POLYFILL_UNSUPPORTED (no cells written) for an H3 row
 * holding a non-finite vertex, or a BNG row without area (searches through the 12 pentagon base
 * cells follow H3's _kRingInternal fallback, as h3-java does).  An empty
 * geometry gives no cells.  Errors: MOSAIC_E_RES, MOSAIC_E_NAN (BNG NaN vertex), MOSAIC_E_CAPACITY. */
#define MOSAIC_POLYFILL_OK 0
#define MOSAIC_POLYFILL_UNSUPPORTED (-2)
typedef struct mosaic_cell_lists mosaic_cell_lists;
int mosaic_polyfill(mosaic_ctx* ctx, int grid, int res, int64_t n_geoms, const int64_t* geom_parts,
                    const int64_t* part_rings, const int64_t* ring_offsets, const double* xy, mosaic_cell_lists** out);
int mosaic_cell_lists_info(const mosaic_cell_lists* lists, int64_t* n_rows, int64_t* n_cells);
/* offsets[n_rows + 1], cells[n_cells], status[n_rows] (any may be null) */
int mosaic_cell_lists_export(const mosaic_cell_lists* lists, int64_t* offsets, int64_t* cells, int32_t* status);
int mosaic_cell_lists_destroy(mosaic_cell_lists* lists);
/* Device time (HIP events on the calling thread's stream) of the calling thread's last mosaic_polyfill, ms. */
double mosaic_polyfill_last_ms(void);

/* getBufferRadius(geometry, res) per geometry (the radius mosaicFill buffers by, core/Mosaic.scala:68):
 * H3 (H3IndexSystem.scala:73-80): the largest distance (degrees) from the centroid of the cell
 * holding the geometry's JTS centroid (its indexToGeometry polygon's JTS centroid) to that polygon's
 * ring points; NaN for a geometry without area.  BNG (BNGIndexSystem.scala:146-149): edge * sqrt(2) / 2.
 * Geometries in the flat-ring layout of mosaic_polyfill; out[n_geoms]. */
int mosaic_buffer_radius(mosaic_ctx* ctx, int grid, int res, int64_t n_geoms, const int64_t* geom_parts,
                         const int64_t* part_rings, const int64_t* ring_offsets, const double* xy, double* out);

/* Execution state of the calling thread on ctx (its device, stream, the "jdk" option and the
 * device's CU count), for the library's own translation units. */
int mosaic_ctx_exec(mosaic_ctx* ctx, int* device, void** stream, int* jdk, int* n_cu);

/* ---- grid_boundaryaswkb over a cell column (BNG) ---- */
/* out[93 i .. 93 i + 92] = the WKB JTS writes for BNGIndexSystem.indexToGeometry(ids[i])
 * (core/index/BNGIndexSystem.scala indexToGeometry; functions/MosaicContext.scala
 * grid_boundaryaswkb -> expressions/index/IndexGeometry.scala:65-75): big-endian 2D Polygon of the
 * cell square, 5 points.  Null rows (valid[i] == 0) are left zero.  H3 cells are served by
 * mosaic_h3_cell_geometry mode 2 (variable-length rings); with grid H3 this entry returns
 * MOSAIC_E_ARG. */
int mosaic_cell_boundary_wkb(mosaic_ctx* ctx, int grid, const int64_t* ids, const uint8_t* valid, int64_t n,
                             uint8_t* out);

#ifdef __cplusplus
}
#endif
#endif
