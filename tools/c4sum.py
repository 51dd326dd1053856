"""Summarise a GPU C4 run directory: kbench lines (ms, tests, pairs) and, when present, the rocprofv3
kernel trace (average ms per kernel).  usage: python tools/c4sum.py gpurun_out/TAG"""
import glob
import json
import os
import sqlite3
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "c4*.txt"))):
    for line in open(f):
        line = line.strip()
        if line.startswith("{"):
            r = json.loads(line)
            if r.get("ms"):
                print(os.path.basename(f), round(r["ms"], 3), "tests", r.get("contains_tests"), "pairs", r.get("pairs"),
                      "exact", r.get("exact_path_rows"), "build_s", r.get("build_s"))
tl = os.path.join(d, "tests.log")
if os.path.exists(tl):
    print([l.strip() for l in open(tl) if "passed" in l or "failed" in l or "error" in l.lower()][-1:])
for st in sorted(glob.glob(os.path.join(d, "stats*.csv"))):
    import csv
    print(os.path.basename(st))
    rows = sorted(csv.DictReader(open(st)), key=lambda r: -float(r["TotalDurationNs"]))[:6]
    for r in rows:
        print(f"  {float(r['AverageNs']) / 1e6:8.3f} ms x{int(r['Calls']):3d}  {r['Name'][:100]}")
for db in glob.glob(os.path.join(d, "prof", "*.db")):
    c = sqlite3.connect(db)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    kt = [t for t in tabs if "kernel_dispatch" in t.lower()][0]
    ks = [t for t in tabs if "kernel_symbol" in t.lower()][0]
    q = (f"select s.kernel_name, count(*), avg(d.end-d.start)/1e6 from {kt} d join {ks} s on d.kernel_id=s.id "
         "group by s.kernel_name order by 3 desc limit 8")
    for name, n, ms in c.execute(q):
        print(f"  {ms:8.3f} ms x{n:3d}  {name[:100]}")
