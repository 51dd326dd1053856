"""Timing of st_intersects_aggregate (mosaic_intersects_aggregate) and of st_intersection_aggregate's
area (mosaic_intersection_aggregate) and geometry (mosaic_intersection_aggregate_geometry: GPU cell
overlay + host stitching into WKB) on the GPU box: the 263 NYC zones chipped at H3 res 9 and 10
joined with a translated copy.  Prints one JSON line per case (groups, true groups, refused groups,
ms for each whole call incl. D2H)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from mosaic_amd import MosaicContext
    from mosaic_amd.context import tessellate
    from mosaic_amd.data import PolygonSet

    ctx = MosaicContext.build("H3")
    for name, res, shift in (("nyc_taxi_zones", 9, (0.0007, -0.0011)), ("nyc_taxi_zones", 10, (0.0007, -0.0011)),
                             ("nyc_taxi_zones", 9, (0.0, 0.0))):
        z = PolygonSet.load(name)
        m = PolygonSet(z.xy + np.array(shift), z.ring_offsets, z.part_rings, z.geom_parts, z.names)
        l, r = tessellate("H3", z, res), tessellate("H3", m, res)
        tl = ctx.chip_table(l["is_core"], l["index_id"], l["wkb"], l["polygon_key"], res)
        tr = ctx.chip_table(r["is_core"], r["index_id"], r["wkb"], r["polygon_key"], res)
        ctx.st_intersects_aggregate(tl, tr)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            lk, rk, fl = ctx.st_intersects_aggregate(tl, tr)
            ts.append((time.perf_counter() - t0) * 1e3)
        ctx.st_intersection_aggregate_area(tl, tr)
        ta = []
        for _ in range(5):
            t0 = time.perf_counter()
            _, _, area, st = ctx.st_intersection_aggregate_area(tl, tr)
            ta.append((time.perf_counter() - t0) * 1e3)
        tg = []
        for _ in range(3):
            t0 = time.perf_counter()
            _, _, garea, gst, wkb = ctx.st_intersection_aggregate(tl, tr)
            tg.append((time.perf_counter() - t0) * 1e3)
        print(json.dumps({"case": f"{name} res {res} shift {shift}", "chips": [len(l["index_id"]), len(r["index_id"])],
                          "groups": int(len(fl)), "true": int(fl.sum()), "ms_median": float(np.median(ts)),
                          "area_ms_median": float(np.median(ta)), "area_refused_groups": int(st.sum()),
                          "area_total": float(area[st == 0].sum()), "geometry_ms_median": float(np.median(tg)),
                          "geometry_refused_groups": int(gst.sum()),
                          "wkb_bytes": int(sum(len(w) for w in wkb if w is not None))}), flush=True)
        tl.close()
        tr.close()


if __name__ == "__main__":
    main()
