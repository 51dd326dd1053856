"""Writes tests/golden/reference_vectors.json: known answers transcribed from the reference's own
tests and docs (and, for H3, from the public H3 documentation), each with its source.

The reference (Scala/Spark + H3/JTS jars) cannot run in this image (no JVM, no jars); these
vectors are data copied from its test files and docs, not code.  Re-run to regenerate:
    python tests/golden/make_reference_vectors.py
"""
import json
import os

H3_POINT_TO_CELL = [
    # lon, lat, res, cell, source
    (30.0, 10.0, 10, 623385352048508927,
     "reference docs/source/api/spatial-indexing.rst:53-58 (grid_longlatascellid) and :132-155"),
    (-74.044444, 40.689167, 10, 0x8A2A1072B59FFFF,
     "uber/h3 README 'Example (C)': latLngToCell(40.689167, -74.044444, 10)"),
    (-122.0553238, 37.3615593, 7, 0x87283472BFFFFFF,
     "uber/h3-js README: h3.latLngToCell(37.3615593, -122.0553238, 7)"),
    (-122.0553238, 37.3615593, 5, 0x85283473FFFFFFF,
     "uber/h3-py docs/tests: geo_to_h3(37.3615593, -122.0553238, 5)"),
    (-122.418307270836, 37.7752702151959, 9, 0x8928308280FFFFF,
     "uber/h3-py README: h3_to_geo('8928308280fffff') centre maps back to its cell"),
]

# reference docs/source/api/spatial-indexing.rst:213-221 (grid_polyfill res 0) and :546-556
# (grid_tessellateexplode res 0) for MULTIPOLYGON (((30 20, 45 40, 10 40, 30 20)),
# ((15 5, 40 10, 10 20, 5 10, 15 5)))
H3_RES0_POLYFILL = [577586652210266111, 578360708396220415, 577269992861466623]
H3_RES0_TESSELLATE = [577481099093999615, 578044049047420927, 578782920861286399, 577023702256844799,
                      577938495931154431, 577586652210266111, 577269992861466623, 578360708396220415]

# src/test/scala/com/databricks/labs/mosaic/core/index/TestBNGIndexSystem.scala
BNG_POINT_TO_INDEX = [
    (538825, 179111, 1, 105010, "TQ"), (538825, 179111, 2, 10501370, "TQ37"),
    (538825, 179111, 3, 1050138790, "TQ3879"), (538825, 179111, 4, 105013887910, "TQ388791"),
    (538825, 179111, 5, 10501388279110, "TQ38827911"), (538825, 179111, 6, 1050138825791110, "TQ3882579111"),
    (538825, 179111, -1, 1050, "T"), (538825, 179111, -2, 105012, "TQNW"),
    (538825, 179111, -3, 10501373, "TQ37NE"), (538825, 179111, -4, 1050138794, "TQ3879SE"),
    (538825, 179111, -5, 105013887911, "TQ388791SW"), (538825, 179111, -6, 10501388279114, "TQ38827911SE"),
]
BNG_SOURCE = "reference src/test/scala/com/databricks/labs/mosaic/core/index/TestBNGIndexSystem.scala:10-90"
# TestBNGIndexSystem.scala:156-161: out-of-range coordinates still encode (isValid false)
BNG_INVALID = [(-50000.0, 50.0, 3), (50.0, 500000000.0, 4)]

# src/test/scala/com/databricks/labs/mosaic/expressions/geometry/ST_ContainsBehaviors.scala:22-36
CONTAINS = {
    "polygon": "POLYGON ((10 10, 110 10, 110 110, 10 110, 10 10), (20 20, 20 30, 30 30, 30 20, 20 20), "
               "(40 20, 40 30, 50 30, 50 20, 40 20))",
    "cases": [["POINT (35 25)", True], ["POINT (25 25)", False]],
    "source": "reference src/test/scala/com/databricks/labs/mosaic/expressions/geometry/ST_ContainsBehaviors.scala:22-36",
}


def main():
    out = {
        "h3_point_to_cell": [dict(lon=a, lat=b, res=r, cell=c, source=s) for a, b, r, c, s in H3_POINT_TO_CELL],
        "h3_res0_polyfill": H3_RES0_POLYFILL,
        "h3_res0_tessellate": H3_RES0_TESSELLATE,
        "h3_res0_source": "reference docs/source/api/spatial-indexing.rst:213-221, 546-556",
        "bng_point_to_index": [dict(e=e, n=n, res=r, id=i, fmt=f) for e, n, r, i, f in BNG_POINT_TO_INDEX],
        "bng_source": BNG_SOURCE,
        "bng_invalid": [dict(e=e, n=n, res=r) for e, n, r in BNG_INVALID],
        "contains": CONTAINS,
    }
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_vectors.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
