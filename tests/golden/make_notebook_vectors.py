"""Writes tests/golden/notebook_vectors.json: the H3 answers the reference's own docs notebooks
print, transcribed as data (inputs + the reference's outputs), never the notebooks themselves.

Sources (all under /root/reference, read as text; the reference cannot run here -- no JVM):
  docs/source/usage/grid-indexes.ipynb
    cell 10  resolution = 9 (MosaicFrame.get_optimal_resolution)
    cell 12  grid_longlatascellid(pickup_longitude, pickup_latitude, 9): 20 trips -> res-9 cells
    cell 16  explode(grid_polyfill(geometry, 9)) for Homecrest (location 123): first rows, in
             h3-java's output order
  docs/source/usage/quickstart.ipynb
    cell 25  grid_longlatascellid(pickup / dropoff lon, lat, 10): 20 trips x 2 points -> res-10 cells
    cell 26  explode(grid_polyfill(geometry, 10)) for Freshkills Park (location 99), in order
    cell 32  displayMosaic(grid_tessellateexplode(geometry, 10)): 1,000 chip rows (zone, is_core,
             index_id, base64 little-endian WKB of border chips; core chips carry no geometry)
    cell 38  the chip join's first 20 rows (pickup point, pickup_h3, zone, is_core, chip index_id)
             -- the notebook's filter is `~is_core | st_contains(...)`, so every shown row is a
             border chip whose cell equals the pickup cell
  docs/source/usage/kepler.ipynb
    cell 10  the first zone's geometry (GeoJSON) and
    cell 27  its grid_tessellateexplode(geom, 9) chips as (index_id, WKT): core chips carry the
             cell polygon (h3ToGeoBoundary, JTS WKTWriter digits = Java Double.toString)

The writer runs here only (it reads /root/reference); the JSON it writes is what tests load.
    python tests/golden/make_notebook_vectors.py
"""
import base64
import html
import json
import os
import re

REF = "/root/reference/docs/source/usage"


def _cell_html(nb, cell, output=0):
    d = json.load(open(os.path.join(REF, nb)))
    data = d["cells"][cell]["outputs"][output]["data"]["text/html"]
    return "".join(data) if isinstance(data, list) else data


def _ansi_table(nb, cell):
    """Spark df.show() text inside the cell's ansiout div -> list of dict rows."""
    s = _cell_html(nb, cell)
    s = html.unescape(s[s.index('<div class="ansiout">') + len('<div class="ansiout">'):])
    lines = [ln for ln in s.split("\n") if ln.strip()]
    rows, header = [], None
    for ln in lines:
        if ln.startswith("+") or ln.startswith("only showing") or ln.startswith("</div>"):
            continue
        fields = [f.strip() for f in ln.rstrip().rstrip("|").split("|")]
        if header is None:
            header = fields
            continue
        if len(fields) != len(header):
            continue
        rows.append(dict(zip(header, fields)))
    return rows


def _kepler_datasets(nb, cell, output):
    s = _cell_html(nb, cell, output)
    out = []
    dec = json.JSONDecoder()
    for m in re.finditer(r'"columns": \[([^\]]*)\], "data": ', s):
        cols = json.loads("[" + m.group(1) + "]")
        arr, _ = dec.raw_decode(s[m.end():])
        out.append((cols, arr))
    return out


def _html_table(nb, cell):
    s = _cell_html(nb, cell)
    head = re.findall(r"<th>(.*?)</th>", s, re.S)
    rows = []
    for r in re.findall(r"<tr>(.*?)</tr>", s, re.S):
        tds = re.findall(r"<td>(.*?)</td>", r, re.S)
        if tds:
            rows.append(dict(zip(head, [html.unescape(t) for t in tds])))
    return rows


def main():
    out = {"source": "reference docs notebooks (docs/source/usage/*.ipynb), outputs transcribed as data"}

    res = re.search(r"Out\[\d+\]: (\d+)", _cell_html("grid-indexes.ipynb", 10)).group(1)
    assert res == "9"
    out["grid_indexes_points_res9"] = {
        "source": "docs/source/usage/grid-indexes.ipynb cell 12 (grid_longlatascellid, resolution from cell 10)",
        "res": 9,
        "rows": [[r["pickup_longitude"], r["pickup_latitude"], int(r["ix"])]
                 for r in _ansi_table("grid-indexes.ipynb", 12)],
    }
    out["homecrest_polyfill_res9"] = {
        "source": "docs/source/usage/grid-indexes.ipynb cell 16 (explode(grid_polyfill(geometry, 9))), shown prefix",
        "zone": "Homecrest", "location_id": 123, "res": 9,
        "cells": [int(r["ix"]) for r in _ansi_table("grid-indexes.ipynb", 16) if r["zone"] == "Homecrest"],
    }
    pts = []
    for r in _ansi_table("quickstart.ipynb", 25):
        pts.append([r["pickup_longitude"], r["pickup_latitude"], int(r["pickup_h3"])])
        pts.append([r["dropoff_longitude"], r["dropoff_latitude"], int(r["dropoff_h3"])])
    out["quickstart_points_res10"] = {
        "source": "docs/source/usage/quickstart.ipynb cell 25 (grid_longlatascellid pickup and dropoff, res 10)",
        "res": 10, "rows": pts,
    }
    out["freshkills_polyfill_res10"] = {
        "source": "docs/source/usage/quickstart.ipynb cell 26 (explode(grid_polyfill(geometry, 10))), shown prefix",
        "zone": "Freshkills Park", "location_id": 99, "res": 10,
        "cells": [int(r["h3"]) for r in _ansi_table("quickstart.ipynb", 26) if r["zone"] == "Freshkills Park"],
    }
    chips = []
    for r in _html_table("quickstart.ipynb", 32):
        w = r["wkb"]
        chips.append([r["zone"], int(r["location_id"]), r["is_core"] == "true", int(r["h3"]),
                      None if w == "null" else base64.b64decode(w).hex()])
    out["quickstart_tessellation_res10"] = {
        "source": "docs/source/usage/quickstart.ipynb cell 32 (displayMosaic of grid_tessellateexplode(geometry, 10)): "
                  "the first 1,000 rows; [zone, location_id, is_core, index_id, wkb hex (little-endian) or null]",
        "res": 10, "rows": chips,
    }
    join = []
    for r in _ansi_table("quickstart.ipynb", 38):
        join.append([r["pickup_longitude"], r["pickup_latitude"], int(r["pickup_h3"]), int(r["location_id"]),
                     r["is_core"] == "true", int(r["h3"])])
    out["quickstart_join_rows_res10"] = {
        "source": "docs/source/usage/quickstart.ipynb cell 38 (join on pickup_h3 == index_id, filter "
                  "~is_core | st_contains): [pickup lon, pickup lat, pickup_h3, location_id, is_core, index_id]",
        "res": 10, "rows": join,
    }
    (cols, geo), = _kepler_datasets("kepler.ipynb", 10, 2)
    g = json.loads(geo[0][cols.index("geom_json")])
    (cols, kchips), = _kepler_datasets("kepler.ipynb", 27, 2)
    out["kepler_tessellation_res9"] = {
        "source": "docs/source/usage/kepler.ipynb cell 10 (geometry of neighbourhoods.limit(1)) and cell 27 "
                  "(grid_tessellateexplode(geom, 9) chips as WKT); [index_id, wkt]",
        "res": 9, "geometry": g, "rows": [[int(a), b] for a, b in kchips],
    }
    # location_id of each feature of notebooks/data/NYC_Taxi_Zones.geojson, in the order of the
    # nyc_taxi_zones.npz fixture (make_fixtures.py keeps the file's feature order)
    with open("/root/reference/notebooks/data/NYC_Taxi_Zones.geojson") as fh:
        feats = [json.loads(line) for line in fh if line.strip()]
    out["nyc_location_ids"] = [int(f["properties"]["location_id"]) for f in feats]
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "notebook_vectors.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=0, separators=(",", ":"))
    print("wrote", path, {k: len(v["rows"] if "rows" in v else v.get("cells", [])) for k, v in out.items()
                         if isinstance(v, dict)})


if __name__ == "__main__":
    main()
