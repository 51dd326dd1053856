"""rocprofv3 --kernel-trace --stats output (rocpd SQLite database or *_kernel_stats.csv) ->
a compact kernel_stats CSV (name shortened to the kernel's own name and template arguments).

    python tools/prof_summary.py gpurun_out/prof profiles/r02_bench_kernel_stats.csv
"""
import csv
import glob
import os
import sqlite3
import sys


def short(name):
    name = name.replace("void ", "")
    if name.startswith("at::native"):
        return name.split("<", 1)[0] + "<...> (torch)"
    return name.split("(", 1)[0]


def rows_from(path):
    dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    if dbs:
        c = sqlite3.connect(dbs[0])
        return [(short(n), int(calls), float(tot), float(avg), float(pct))
                for n, calls, tot, avg, pct in c.execute("select name, total_calls, total_duration, average, percentage "
                                                         "from top_kernels")]
    out = []
    for f in glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                out.append((short(r["Name"]), int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]),
                            float(r["Percentage"])))
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    rows = rows_from(src)
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
        for r in rows:
            w.writerow([r[0], r[1], round(r[2], 3), round(r[3], 3), round(r[4], 3)])
    print(open(dst).read())


if __name__ == "__main__":
    main()
