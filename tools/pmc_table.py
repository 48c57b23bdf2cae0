"""Mean per-dispatch counter values by kernel from a rocprofv3 --pmc run.

    python tools/pmc_table.py <output dir> [kernel substring]
"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
vals = collections.defaultdict(lambda: collections.defaultdict(dict))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            k = r["Kernel_Name"]
            if pat in k:
                d = vals[k][r["Correlation_Id"]]
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k, disp in vals.items():
    names = sorted({c for d in disp.values() for c in d})
    n = len(disp)
    means = {c: sum(d.get(c, 0.0) for d in disp.values()) / n for c in names}
    print(f"{k[:60]} ({n} dispatches): " + ", ".join(f"{c}={v:.4g}" for c, v in means.items()))
