"""Overlap of uploads, kernels and downloads in a rocprofv3 trace.

Reads ``<dir>/<prefix>_kernel_trace.csv`` and ``_memory_copy_trace.csv``
(``rocprofv3 --kernel-trace --memory-copy-trace --output-format csv``),
splits the operations into calls at host gaps longer than ``--gap-ms`` and
reports, per call: its span, the busy time of each engine class (H2D copies,
kernels, D2H copies), the time two or three classes were active at once, and
a one-line text timeline.  ``--names`` labels the LAST calls in order (the
calls before them are calibration and warm-up).

    python tools/overlap_timeline.py gpurun_out/prof_overlap \\
        --names 3phase,event_b8,event_b8_4streams,driver_b8_q4,driver_b8_q16
"""
import argparse
import csv
import glob
import json
import os


def load(d):
    ops = []
    for f in glob.glob(os.path.join(d, "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            ops.append(("K", int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    for f in glob.glob(os.path.join(d, "*memory_copy_trace.csv")):
        for r in csv.DictReader(open(f)):
            kind = "U" if "HOST_TO_DEVICE" in r["Direction"] else "D" if "DEVICE_TO_HOST" in r["Direction"] else "X"
            ops.append((kind, int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"]))
    ops.sort(key=lambda o: o[1])
    return ops


def union(iv):
    out = []
    for b, e in sorted(iv):
        if out and b <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([b, e])
    return out


def measure(iv):
    return sum(e - b for b, e in iv)


def intersect(a, b):
    i = j = 0
    out = []
    while i < len(a) and j < len(b):
        lo, hi = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if lo < hi:
            out.append([lo, hi])
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def call_stats(ops, width=72):
    t0, t1 = min(o[1] for o in ops), max(o[2] for o in ops)
    cls = {k: union([(o[1], o[2]) for o in ops if o[0] == k]) for k in "UKD"}
    ku, kd, ud = intersect(cls["K"], cls["U"]), intersect(cls["K"], cls["D"]), intersect(cls["U"], cls["D"])
    all3 = intersect(ku, cls["D"])
    line = []
    for c in range(width):
        a, b = t0 + (t1 - t0) * c / width, t0 + (t1 - t0) * (c + 1) / width
        act = "".join(k for k in "UKD" if any(lo < b and hi > a for lo, hi in cls[k]))
        line.append({"": ".", "U": "u", "K": "k", "D": "d", "UK": "1", "KD": "2", "UD": "x", "UKD": "3"}[act])
    ms = lambda ns: round(ns / 1e6, 3)  # noqa: E731
    return {"span_ms": ms(t1 - t0), "h2d_ms": ms(measure(cls["U"])), "kernel_ms": ms(measure(cls["K"])),
            "d2h_ms": ms(measure(cls["D"])), "kernel_and_h2d_ms": ms(measure(ku)), "kernel_and_d2h_ms": ms(measure(kd)),
            "h2d_and_d2h_ms": ms(measure(ud)), "all_three_ms": ms(measure(all3)),
            "ops": {k: sum(1 for o in ops if o[0] == k) for k in "UKD"}, "timeline": "".join(line)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--gap-ms", type=float, default=5.0)
    ap.add_argument("--names", default="")
    ap.add_argument("--min-ops", type=int, default=3)
    a = ap.parse_args()
    ops = [o for o in load(a.dir) if o[0] in "UKD"]
    calls, cur = [], []
    for o in ops:
        if cur and o[1] - max(c[2] for c in cur) > a.gap_ms * 1e6:
            calls.append(cur)
            cur = []
        cur.append(o)
    if cur:
        calls.append(cur)
    calls = [c for c in calls if len(c) >= a.min_ops]
    names = [n for n in a.names.split(",") if n]
    out = {}
    for i, c in enumerate(calls[-len(names):] if names else calls):
        out[names[i] if names else f"call{i}"] = call_stats(c)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
