"""Projects the London postcode zones (the reference's notebooks/data/London_Postcode_Zones.geojson,
EPSG:4326, packed in london_postcode_zones.npz) once to British National Grid metres (EPSG:27700)
for the C5 config ("the London postcodes projected once to EPSG:27700 by the fixture
generator ... the projected coordinates are committed so both sides see identical inputs").

Written out in numpy (no pyproj in the image): WGS84 geodetic -> ECEF -> the 7-parameter Helmert
WGS84 -> OSGB36 (the Ordnance Survey's published parameters: tx -446.448 m, ty +125.157 m,
tz -542.060 m, scale +20.4894 ppm, rx -0.1502", ry -0.2470", rz -0.8421"; ~5 m accuracy, the
EPSG:1314 inverse) -> geodetic on Airy 1830 -> Transverse Mercator of the National Grid
(F0 0.9996012717, true origin 49 N 2 W, false origin E 400000 m, N -100000 m), the OS guide's
series.  The projection is not on the hot path; what matters is that the fixture is deterministic
and committed.

    python tests/golden/make_bng_fixture.py   ->  tests/golden/london_postcodes_bng.npz
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def wgs84_to_osgb36(lon_deg, lat_deg):
    lat = np.radians(lat_deg)
    lon = np.radians(lon_deg)
    a, b = 6378137.000, 6356752.3141  # GRS80 / WGS84
    e2 = 1.0 - (b * b) / (a * a)
    nu = a / np.sqrt(1.0 - e2 * np.sin(lat) ** 2)
    x = nu * np.cos(lat) * np.cos(lon)
    y = nu * np.cos(lat) * np.sin(lon)
    z = (1.0 - e2) * nu * np.sin(lat)
    tx, ty, tz = -446.448, 125.157, -542.060
    s = 20.4894e-6
    rx, ry, rz = (np.radians(v / 3600.0) for v in (-0.1502, -0.2470, -0.8421))
    x2 = tx + (1.0 + s) * x + (-rz) * y + ry * z
    y2 = ty + rz * x + (1.0 + s) * y + (-rx) * z
    z2 = tz + (-ry) * x + rx * y + (1.0 + s) * z
    a2, b2 = 6377563.396, 6356256.909  # Airy 1830
    e22 = 1.0 - (b2 * b2) / (a2 * a2)
    p = np.sqrt(x2 * x2 + y2 * y2)
    phi = np.arctan2(z2, p * (1.0 - e22))
    for _ in range(10):
        nu2 = a2 / np.sqrt(1.0 - e22 * np.sin(phi) ** 2)
        phi = np.arctan2(z2 + e22 * nu2 * np.sin(phi), p)
    lam = np.arctan2(y2, x2)
    return lam, phi


def osgb36_to_grid(lam, phi):
    a, b = 6377563.396, 6356256.909
    F0 = 0.9996012717
    lat0, lon0 = np.radians(49.0), np.radians(-2.0)
    N0, E0 = -100000.0, 400000.0
    e2 = 1.0 - (b * b) / (a * a)
    n = (a - b) / (a + b)
    sp, cp, tp = np.sin(phi), np.cos(phi), np.tan(phi)
    nu = a * F0 / np.sqrt(1.0 - e2 * sp * sp)
    rho = a * F0 * (1.0 - e2) / (1.0 - e2 * sp * sp) ** 1.5
    eta2 = nu / rho - 1.0
    dphi, sphi = phi - lat0, phi + lat0
    M = b * F0 * ((1.0 + n + 1.25 * n ** 2 + 1.25 * n ** 3) * dphi
                  - (3.0 * n + 3.0 * n ** 2 + 2.625 * n ** 3) * np.sin(dphi) * np.cos(sphi)
                  + (1.875 * n ** 2 + 1.875 * n ** 3) * np.sin(2.0 * dphi) * np.cos(2.0 * sphi)
                  - (35.0 / 24.0) * n ** 3 * np.sin(3.0 * dphi) * np.cos(3.0 * sphi))
    I = M + N0
    II = nu / 2.0 * sp * cp
    III = nu / 24.0 * sp * cp ** 3 * (5.0 - tp ** 2 + 9.0 * eta2)
    IIIA = nu / 720.0 * sp * cp ** 5 * (61.0 - 58.0 * tp ** 2 + tp ** 4)
    IV = nu * cp
    V = nu / 6.0 * cp ** 3 * (nu / rho - tp ** 2)
    VI = nu / 120.0 * cp ** 5 * (5.0 - 18.0 * tp ** 2 + tp ** 4 + 14.0 * eta2 - 58.0 * tp ** 2 * eta2)
    dl = lam - lon0
    N = I + II * dl ** 2 + III * dl ** 4 + IIIA * dl ** 6
    E = E0 + IV * dl + V * dl ** 3 + VI * dl ** 5
    return E, N


def project(lon, lat):
    lam, phi = wgs84_to_osgb36(lon, lat)
    return osgb36_to_grid(lam, phi)


def main():
    z = np.load(os.path.join(HERE, "london_postcode_zones.npz"), allow_pickle=False)
    xy = z["xy"]
    e, n = project(xy[:, 0], xy[:, 1])
    out = np.stack([e, n], axis=1)
    # rings stay closed exactly: first == last in the source, and the map is a function
    np.savez_compressed(os.path.join(HERE, "london_postcodes_bng.npz"), xy=out, ring_offsets=z["ring_offsets"],
                        part_rings=z["part_rings"], geom_parts=z["geom_parts"], names=z["names"])
    print(f"{len(z['geom_parts']) - 1} zones, {len(xy)} vertices, E [{e.min():.1f}, {e.max():.1f}], "
          f"N [{n.min():.1f}, {n.max():.1f}]")


if __name__ == "__main__":
    main()
