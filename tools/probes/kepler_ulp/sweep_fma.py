"""Exact-ring counts for run_fma.sh (same scoring as sweep.py)."""
import json
import math
import re
import subprocess
import sys

w, vectors = sys.argv[1], sys.argv[2]
rows = json.load(open(vectors))["kepler_tessellation_res9"]["rows"]
num = re.compile(r"-?\d+\.?\d*(?:[eE][-+]?\d+)?")
ref = {}
for cid, wkt in rows:
    if wkt.count("(") > 2:
        continue
    v = [float(t) for t in num.findall(wkt)]
    ref[cid] = list(zip(v[0::2], v[1::2]))
cells = " ".join(str(c) for c in ref)


def run(drv, args):
    out = subprocess.run([drv] + [str(a) for a in args], input=cells, capture_output=True, text=True).stdout
    res = {}
    for line in out.split("\n"):
        if line:
            t = line.split()
            v = [float.fromhex(x) * 180.0 / math.pi for x in t[2:]]
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


modes = {0: "H3 x87 steps (oracle)", 4: "H3 double constants", 5: "H3 binary128 + FMA (a*b first)",
         6: "H3 binary128 + FMA (c*d*e first)", 7: "H3 binary128, no FMA"}
for lib in ("nocontract", "contract"):
    for m, name in modes.items():
        e = exact(run(f"{w}/drv_{lib}", [m, 32]))
        print("libm restatement %-10s + %-36s exact %d of %d" % (lib, name, *e))
