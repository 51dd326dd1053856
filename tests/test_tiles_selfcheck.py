"""CPU-only: the H3 tile directory and point raster (mosaic_amd/csrc/tiles.h, tiles_build.cpp)
compiled for the host.  The directory gives, for every point it certifies, the chip-table slot of
the point's exact H3 cell (h3_exact, the oracle's restatement) -- and "skip" only for points whose
exact cell carries no chip.  Every pure point-raster code equals the exact answer (core chips of
the exact cell + border chips whose JTS contains holds).  Tessellated NYC zones at several
resolutions (uniform points, points on / next to tile lines, chip vertices and chip segments),
plus synthetic cell sets near icosahedron face edges, pentagons, high latitudes and the
antimeridian (where the builder must either decline or stay exact)."""
import os
import re
import struct
import subprocess

import numpy as np
import pytest

import oracle
from mosaic_amd.context import tessellate
from mosaic_amd.data import PolygonSet

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = tmp_path_factory.mktemp("tiles") / "tiles_sc"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-Wno-unknown-pragmas", "-pthread", "-o", str(out),
                    os.path.join(ROOT, "tests", "native", "tiles_selfcheck.cpp")], check=True)
    return out


def _run(exe, tmp_path, res, chips, npts=300_000, seed=3, sc=(16, 8)):
    path = tmp_path / f"chips_{res}.bin"
    offs, data = chips["wkb"]
    with open(path, "wb") as f:
        f.write(struct.pack("<iI", res, len(chips["index_id"])))
        for i in range(len(chips["index_id"])):
            w = bytes(data[offs[i]:offs[i + 1]])
            f.write(struct.pack("<qBiI", int(chips["index_id"][i]), int(chips["is_core"][i]),
                                int(chips["polygon_key"][i]), len(w)))
            f.write(w)
    out = subprocess.run([str(exe), str(path), str(npts), str(seed), str(sc[0]), str(sc[1])], check=True,
                         capture_output=True, text=True)
    built, bad, checked, skipped, full, unc, miss, rbuilt, rbad, rpure, rmixed = map(int, out.stdout.split())
    return dict(built=built, bad=bad, checked=checked, skipped=skipped, full=full, unc=unc, miss=miss,
                raster=rbuilt, raster_bad=rbad, raster_pure=rpure, raster_mixed=rmixed, log=out.stderr)


@pytest.mark.parametrize("res,sc", [(7, (16, 8)), (8, (8, 4)), (9, (32, 16)), (9, (16, 8)), (9, (4, 2)),
                                    (10, (16, 8)), (11, (8, 8))])
def test_tiles_nyc_tessellation(exe, tmp_path, res, sc):
    zones = PolygonSet.load("nyc_taxi_zones_35" if res >= 10 else "nyc_taxi_zones")
    chips = tessellate("H3", zones, res)
    r = _run(exe, tmp_path, res, chips, sc=sc)
    assert r["built"] == 1, r["log"]
    assert r["bad"] == 0, r["log"]
    assert r["checked"] > 200_000
    assert r["miss"] == 0
    assert r["raster"] == 1, r["log"]
    assert r["raster_bad"] == 0, r["log"]
    assert r["raster_pure"] > 0.4 * 300_000
    # k_join_stream_pipe's fixed-point lookup (tiles::raster_code_fixed; its pure codes are checked
    # against the exact answer like the float form's) decides as many points
    m = re.search(r"pure codes: float form (\d+), fixed-point form (\d+)", r["log"])
    assert m and int(m.group(2)) >= 0.999 * int(m.group(1)), r["log"]
    # line records in the tile frame: one copy per tile and edge (no duplicates within a tile, and
    # sub-blocks along one edge share a record)
    m = re.search(r"line records (\d+) for (\d+) line sub-blocks, duplicates (\d+)", r["log"])
    assert m and int(m.group(3)) == 0, r["log"]
    if int(m.group(2)) > 20_000:
        assert int(m.group(1)) < 0.9 * int(m.group(2)), r["log"]


def _disc_chips(lon, lat, radius_deg, res, n=20000, seed=0):
    """Core chips (no geometry) for the cells of a disc, with a few polygon keys so that
    neighbouring cells differ: exercises the raster's hexagon-boundary classification."""
    rng = np.random.default_rng(seed)
    x = lon + (rng.random(n) - 0.5) * 2 * radius_deg
    y = np.clip(lat + (rng.random(n) - 0.5) * 2 * radius_deg, -89.9, 89.9)
    cells = np.unique(oracle.h3_point_to_index(x, y, res))
    cells = cells[cells != 0]
    keys = (cells % 5).astype(np.int32)
    return dict(index_id=cells, is_core=np.ones(len(cells), np.uint8), polygon_key=keys,
                wkb=(np.zeros(len(cells) + 1, np.int64), np.zeros(0, np.uint8)))


# (lon, lat, radius, res): a face edge crossing (lon -45 between faces 1 / 6 region), a pentagon
# base cell centre (base cell 4 at about 64.7 N, 10.5 E), Reykjavik-like high latitude, the
# antimeridian, the equator at the prime meridian, a coarse resolution with huge cells.
CASES = [(-45.0, 46.0, 1.5, 7), (10.536199, 64.7, 0.4, 6), (-21.9, 64.1, 0.3, 9), (179.95, -16.5, 0.2, 8),
         (0.0, 0.0, 0.5, 8), (-74.0, 40.7, 3.0, 3), (139.7, 35.7, 0.05, 12)]


@pytest.mark.parametrize("lon,lat,radius,res", CASES)
def test_tiles_synthetic_regions(exe, tmp_path, lon, lat, radius, res):
    r = _run(exe, tmp_path, res, _disc_chips(lon, lat, radius, res), npts=200_000)
    assert r["bad"] == 0, r["log"]
    assert r["raster_bad"] == 0, r["log"]
    if r["built"]:
        assert r["checked"] > 0 and r["raster"] == 1


def test_tile_map_bounds(tmp_path):
    """the closed-form bounds behind the certification (tiles.h TileCurv, rect_tol): on ~3,000
    random tiles (res 3-15, latitudes +-75) the finite-difference |F'|, |F''| along lon / lat lines
    and along random directions stay under jac / kax / kdir, and sampled points of random
    sub-rectangles lie within rect_tol of their corner quadrilateral"""
    exe = tmp_path / "tcc"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-Wno-unknown-pragmas", "-pthread", "-o", str(exe),
                    os.path.join(ROOT, "tests", "native", "tile_curv_check.cpp")], check=True)
    out = subprocess.run([str(exe), "3000"], check=True, capture_output=True, text=True).stdout.split()
    checked, bad = int(out[0]), int(out[1])
    r_jac, r_ax, r_dir, r_rect = map(float, out[2:])
    assert checked > 2500 and bad == 0
    assert r_jac <= 1.0 and r_ax <= 1.0 and r_dir <= 1.0 and r_rect <= 1.0
    # and not vacuous: the first-derivative bound is attained (radial direction), the others within 3x
    assert r_jac > 0.9 and r_ax > 0.3 and r_rect > 0.1


def test_ring_walks_match_jts(tmp_path):
    """CPU: the tile join's ring walks (ring_walk.h: branch-free with its filter fallback, and the
    exact walk) equal JTS locateInRing == INTERIOR (pip_device.h) on ~1.1 M adversarial cases, and
    the certified f32 walk equals it wherever it decides"""
    root = ROOT
    exe = tmp_path / "rwc"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(root, "mosaic_amd", "csrc"),
                    "-o", str(exe), os.path.join(root, "tests", "native", "ring_walk_check.cpp")], check=True)
    cases, bad, f32_cases, f32_undecided, f32_random, f32_random_undecided = map(
        int, subprocess.run([str(exe), "20000"], check=True, capture_output=True, text=True).stdout.split())
    assert cases > 1_000_000 and bad == 0
    # the f32 walk leaves the boundary cases undecided (vertices, points on edges and on rays
    # through vertices: most adversarial points) and decides nearly every random point
    assert f32_cases > 500_000 and f32_random > 100_000 and f32_random_undecided < 1e-3 * f32_random


def test_tile_images(tmp_path):
    """CPU: the binned join's tile images (tile_images.h) for 20k C4-style buildings at H3 res 11
    and the NYC zones at res 10 -- image headers and chip records equal the chip table, and every
    window chip whose envelope holds a point of the tile (random tile points, tile edges, envelope
    corners and edge midpoints) is listed in the point's envelope-raster cell of its part's image as
    k_join_tiles computes it, with the record's cover bit set exactly for non-empty cells"""
    from mosaic_amd.data import synthetic_buildings
    exe = tmp_path / "tic"
    # (sanitized: an out-of-range index in the builder or the keygen arithmetic fails the run)
    subprocess.run(["g++", "-O1", "-std=c++17", "-ffp-contract=off", "-Wno-unknown-pragmas", "-pthread",
                    "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-o", str(exe),
                    os.path.join(ROOT, "tests", "native", "tile_images_check.cpp")], check=True)
    for name, polys, res, cap in (("bld", synthetic_buildings(20000), 11, None),
                                  ("bld_split", synthetic_buildings(20000, sigma=0.0005), 11, 1024),
                                  ("nyc", PolygonSet.load("nyc_taxi_zones_35"), 10, None)):
        chips = tessellate("H3", polys, res)
        path = tmp_path / f"{name}.bin"
        offs, data = chips["wkb"]
        with open(path, "wb") as f:
            f.write(struct.pack("<iI", res, len(chips["index_id"])))
            for i in range(len(chips["index_id"])):
                w = bytes(data[offs[i]:offs[i + 1]])
                f.write(struct.pack("<qBiI", int(chips["index_id"][i]), int(chips["is_core"][i]),
                                    int(chips["polygon_key"][i]), len(w)))
                f.write(w)
        args = [str(exe), str(path), "32"] + ([str(cap)] if cap else [])
        out = subprocess.run(args, check=True, capture_output=True, text=True).stdout.split()
        recs, images, checked, bad, lv0, lv1, lv2 = map(int, out)
        assert recs > 100 and images > recs // 2 and checked > 20_000 and bad == 0, (name, out)
        assert lv0 + lv1 + lv2 == recs, (name, out)
        if cap:  # (dense buildings, small images: records split into 2 x 2 and 4 x 4 parts)
            assert lv1 > 0 and lv2 > 0, (name, out)
