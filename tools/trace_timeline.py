"""Print a rocprofv3 kernel + memory-copy trace as one time-ordered table
(µs from the first event): kind, name / direction, start, end, duration,
bytes.  Gaps longer than ``--gap`` µs between consecutive starts are marked.

    python tools/trace_timeline.py <rocprof output dir> [--from US] [--to US] [--gap US]
"""
import argparse
import csv
import glob
import os


def rows(d):
    out = []
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                out.append(("K", r.get("Kernel_Name", "?")[:40], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), 0))
    for path in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                out.append(("C", r.get("Direction", "?"), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                            int(r.get("Bytes", 0) or 0)))
    return sorted(out, key=lambda x: x[2])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--from", dest="lo", type=float, default=0.0)
    ap.add_argument("--to", dest="hi", type=float, default=float("inf"))
    ap.add_argument("--gap", type=float, default=1000.0)
    a = ap.parse_args()
    rs = rows(a.dir)
    if not rs:
        print("no trace rows")
        return
    t0 = rs[0][2]
    prev = None
    print(f"{'kind':4} {'name':40} {'start_us':>10} {'end_us':>10} {'dur_us':>8} {'MiB':>7}")
    for kind, name, s, e, b in rs:
        su, eu = (s - t0) / 1e3, (e - t0) / 1e3
        if su < a.lo or su > a.hi:
            continue
        if prev is not None and su - prev > a.gap:
            print(f"---- gap {su - prev:.0f} us")
        prev = su
        print(f"{kind:4} {name:40} {su:10.1f} {eu:10.1f} {eu - su:8.1f} {b / 2**20:7.1f}")


if __name__ == "__main__":
    main()
