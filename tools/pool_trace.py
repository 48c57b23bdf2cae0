"""Per-queue view of a device-pool run in a rocprofv3 kernel trace
(``--kernel-trace --output-format csv``): the operations are split into
runs at host gaps longer than ``--gap-ms``; for the chosen run (default:
the one with the most user kernels after the first) every queue's kernel
count, busy time (union of its kernel intervals), first start and last end
relative to the run, and the run's span.  ``rocclr`` blit / stream-op
kernels are counted separately.

    python tools/pool_trace.py gpurun_out/prof_tp [--run N]
"""
import argparse
import collections
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--gap-ms", type=float, default=20.0)
    ap.add_argument("--run", type=int, default=-1)
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.dir, "*kernel_trace.csv")):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    runs, cur, end = [], [], 0
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if cur and s - end > a.gap_ms * 1e6:
            runs.append(cur)
            cur = []
        cur.append(r)
        end = max(end, e) if cur[:-1] else e
    if cur:
        runs.append(cur)
    user = [sum(1 for r in run if "rocclr" not in r["Kernel_Name"]) for run in runs]
    idx = a.run if a.run >= 0 else max(range(1, len(runs)), key=lambda i: (user[i], i)) if len(runs) > 1 else 0
    run = runs[idx]
    t0 = min(int(r["Start_Timestamp"]) for r in run)
    t1 = max(int(r["End_Timestamp"]) for r in run)
    per_q = collections.defaultdict(list)
    for r in run:
        per_q[r["Queue_Id"]].append(r)
    out = {"runs": [{"kernels": len(r), "user_kernels": u} for r, u in zip(runs, user)], "run": idx,
           "span_ms": round((t1 - t0) / 1e6, 3), "queues": {}}
    for q, ks in sorted(per_q.items(), key=lambda kv: kv[0]):
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in ks)
        union = []
        for b, e in iv:
            if union and b <= union[-1][1]:
                union[-1][1] = max(union[-1][1], e)
            else:
                union.append([b, e])
        busy = sum(e - b for b, e in union)
        names = collections.Counter("rocclr" if "rocclr" in r["Kernel_Name"] else "user" for r in ks)
        out["queues"][q] = {"kernels": dict(names), "busy_ms": round(busy / 1e6, 3),
                            "first_ms": round((iv[0][0] - t0) / 1e6, 3), "last_ms": round((max(e for _, e in iv) - t0) / 1e6, 3),
                            "busy_fraction_of_span": round(busy / max(1, t1 - t0), 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
