"""Summarise rocprofv3 output (CSV, or the rocpd SQLite ``*_results.db``;
kernel trace + counters) into markdown.

usage: python tools/summarize_prof.py <rocprof dir> [title] > profiles/<name>.md
"""
import csv
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(d.rstrip("/"))
    print(f"# {title}\n")
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    db = glob.glob(os.path.join(d, "**", "*results.db"), recursive=True)
    per = defaultdict(list)
    if kt:
        for r in csv.DictReader(open(kt[0])):
            per[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    elif db:
        con = sqlite3.connect(db[0])
        for name, dur in con.execute("select name, duration from kernels"):
            per[name].append(dur / 1e3)
    if per:
        print("## Kernel trace (µs per dispatch)\n")
        print("| kernel | calls | mean µs | min µs | max µs | total µs |")
        print("|---|---|---|---|---|---|")
        for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
            print(f"| `{k[:70]}` | {len(v)} | {sum(v)/len(v):.1f} | {min(v):.1f} | {max(v):.1f} | {sum(v):.1f} |")
        print()
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if cc:
        agg = defaultdict(dict)
        names = {}
        for r in csv.DictReader(open(cc[0])):
            key = int(r["Dispatch_Id"])
            names[key] = r["Kernel_Name"]
            agg[key][r["Counter_Name"]] = float(r["Counter_Value"])
        counters = sorted({c for v in agg.values() for c in v})
        print("## Counters per dispatch\n")
        print("| dispatch | kernel | " + " | ".join(counters) + " | L2 hit % |")
        print("|---" * (len(counters) + 3) + "|")
        for k in sorted(agg):
            v = agg[k]
            h, m = v.get("TCC_HIT_sum", 0), v.get("TCC_MISS_sum", 0)
            hit = f"{100*h/(h+m):.1f}" if h + m else "-"
            print(f"| {k} | `{names[k][:40]}` | " + " | ".join(f"{v.get(c, 0):.4g}" for c in counters) + f" | {hit} |")


if __name__ == "__main__":
    main()
