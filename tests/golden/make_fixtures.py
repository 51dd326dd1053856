"""Converts the reference's geometry data files into compact .npz fixtures (data only).

Sources (read here; /root/reference does not exist on the GPU box):
  notebooks/data/NYC_Taxi_Zones.geojson         263 zones (Quickstart polygons; C1-C3)
  src/test/resources/NYC_Taxi_Zones.geojson     35 zones  (MosaicFrameBehaviors join test)
  src/test/resources/nyctaxi_yellow_trips.csv   98 trips  (pickup_longitude / pickup_latitude)
  notebooks/data/London_Postcode_Zones.geojson  177 polygons (BNG config C5)
Output layout per polygon set (all int64 offsets):
  xy [V,2] float64, ring_offsets [R+1], part_rings [P+1], geom_parts [G+1], names [G]
Run:  python tests/golden/make_fixtures.py
"""
import csv
import json
import os

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _features(path):
    with open(path) as fh:
        txt = fh.read().strip()
    if txt.startswith("{") and '"FeatureCollection"' in txt[:200]:
        return json.loads(txt)["features"]
    return [json.loads(line) for line in txt.splitlines() if line.strip()]


def pack(features, name_key):
    xy, ring_offsets, part_rings, geom_parts, names = [], [0], [0], [0], []
    for f in features:
        g = f["geometry"]
        polys = g["coordinates"] if g["type"] == "MultiPolygon" else [g["coordinates"]]
        for poly in polys:
            for ring in poly:
                xy.extend((float(p[0]), float(p[1])) for p in ring)
                ring_offsets.append(len(xy))
            part_rings.append(len(ring_offsets) - 1)
        geom_parts.append(len(part_rings) - 1)
        names.append(str(f["properties"].get(name_key, "")))
    return dict(xy=np.asarray(xy, np.float64), ring_offsets=np.asarray(ring_offsets, np.int64),
                part_rings=np.asarray(part_rings, np.int64), geom_parts=np.asarray(geom_parts, np.int64),
                names=np.asarray(names))


def main():
    nyc = pack(_features(f"{REF}/notebooks/data/NYC_Taxi_Zones.geojson"), "zone")
    np.savez_compressed(os.path.join(OUT, "nyc_taxi_zones.npz"), **nyc)
    nyc35 = pack(_features(f"{REF}/src/test/resources/NYC_Taxi_Zones.geojson"), "zone")
    np.savez_compressed(os.path.join(OUT, "nyc_taxi_zones_35.npz"), **nyc35)
    london = pack(_features(f"{REF}/notebooks/data/London_Postcode_Zones.geojson"), "Name")
    np.savez_compressed(os.path.join(OUT, "london_postcode_zones.npz"), **london)
    with open(f"{REF}/src/test/resources/nyctaxi_yellow_trips.csv") as fh:
        rows = list(csv.DictReader(fh))
    trips = np.array([[float(r["pickup_longitude"]), float(r["pickup_latitude"])] for r in rows], np.float64)
    np.save(os.path.join(OUT, "nyctaxi_yellow_trips_pickups.npy"), trips)
    for k, v in (("nyc", nyc), ("nyc35", nyc35), ("london", london)):
        print(k, "geoms", len(v["geom_parts"]) - 1, "parts", len(v["part_rings"]) - 1, "rings",
              len(v["ring_offsets"]) - 1, "vertices", len(v["xy"]))
    print("trips", trips.shape)


if __name__ == "__main__":
    main()
