"""Exact-ring counts of h3ToGeoBoundary variants against kepler.ipynb cell 27 (see run.sh)."""
import json
import math
import re
import subprocess
import sys

drv, vectors = sys.argv[1], sys.argv[2]
rows = json.load(open(vectors))["kepler_tessellation_res9"]["rows"]
num = re.compile(r"-?\d+\.?\d*(?:[eE][-+]?\d+)?")
ref = {}
for cid, wkt in rows:
    if wkt.count("(") > 2:
        continue
    v = [float(t) for t in num.findall(wkt)]
    ref[cid] = list(zip(v[0::2], v[1::2]))
cells = " ".join(str(c) for c in ref)


def run(args, conv=lambda x: x * 180.0 / math.pi):
    out = subprocess.run([drv] + [str(a) for a in args], input=cells, capture_output=True, text=True).stdout
    res = {}
    for line in out.split("\n"):
        if line:
            t = line.split()
            v = [conv(float.fromhex(x)) for x in t[2:]]
            res[int(t[0])] = list(zip(v[0::2], v[1::2]))
    return res


def ring_ulps(r, want):
    r = r[:-1]
    if len(r) != len(want):
        return None
    return min(max(abs(a - b) / math.ulp(b) for p, q in zip(r[k:] + r[:k], want) for a, b in zip(p, q))
               for k in range(len(r)))


def exact(got):
    us = [ring_ulps(ref[c], got[c]) for c in ref]
    us = [u for u in us if u is not None and u < 100]
    return sum(u == 0 for u in us), len(us)


modes = {0: "oracle (x87 long double steps, glibc 2.35)", 1: "x87 excess precision through r", 3: "x87 through the sqrt7 loop only",
         4: "double constants", 5: "binary128 long double + FMA (a*b first)", 6: "binary128 + FMA (c*d*e first)",
         7: "binary128 long double, no FMA"}
for m, name in modes.items():
    print("%-48s exact %d of %d" % (name, *exact(run([m]))))
fns = ["atan", "atan2", "sin", "cos", "asin"]
best = max(exact(run([0, cr]))[0] for cr in range(1, 32))
print("%-48s best exact %d (31 subsets)" % ("correctly rounded libm subsets", best))
for name, args in [("r +1 ulp", [0, 0, 1]), ("r -1 ulp", [0, 0, -1]), ("atan(r) +1 ulp", [0, 0, 0, 1]),
                   ("atan(r) -1 ulp", [0, 0, 0, -1]), ("azimuth +1 ulp", [0, 0, 0, 0, 1]), ("azimuth -1 ulp", [0, 0, 0, 0, -1])]:
    print("%-48s exact %d of %d" % (name, *exact(run(args))))
for name, conv in [("toDegrees x * (180 / PI) (JDK 9+)", lambda x: x * (180.0 / math.pi)),
                   ("x / (PI / 180)", lambda x: x / (math.pi / 180.0))]:
    print("%-48s exact %d of %d" % (name, *exact(run([0], conv))))
