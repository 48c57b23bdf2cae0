"""Gaps between consecutive dispatches of one kernel in a rocprofv3
kernel-trace CSV: how much of a back-to-back step is launch / dependency
gap rather than kernel time.

    python tools/kernel_gaps.py <trace dir or *_kernel_trace.csv> [kernel substring]
"""
import csv
import glob
import os
import statistics
import sys

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "cek_sgemm"
files = [path] if path.endswith(".csv") else glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
rows = []
for f in files:
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if pat in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
durs = [(e - s) / 1e3 for s, e, _ in rows]
gaps = [(rows[i + 1][0] - rows[i][1]) / 1e3 for i in range(len(rows) - 1)]
# back-to-back gaps only (a host sync or another kernel in between shows as > 50 us)
b2b = [g for g in gaps if g < 50]
print(f"{len(rows)} dispatches of *{pat}*: kernel us median {statistics.median(durs):.1f} "
      f"min {min(durs):.1f}; back-to-back gaps ({len(b2b)}) median {statistics.median(b2b) if b2b else 0:.2f} us "
      f"min {min(b2b) if b2b else 0:.2f} max {max(b2b) if b2b else 0:.2f}")
