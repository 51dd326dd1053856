"""Summarise rocprofv3 counter CSVs (tools/pmc_*.sh, tools/gpu_round.sh pmc steps): mean per launch,
per kernel whose name contains `match` (default: the join kernels).

    python tools/pmc_summary.py DIR [match]
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    match = sys.argv[2] if len(sys.argv) > 2 else "k_join"
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        per = defaultdict(float)
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = (row["Kernel_Name"].split("(")[0], row["Dispatch_Id"], row["Counter_Name"])
                per[k] += float(row["Counter_Value"])
        for (kern, _, ctr), v in per.items():
            if match in kern:
                vals[kern][ctr].append(v)
    out = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in vals.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
