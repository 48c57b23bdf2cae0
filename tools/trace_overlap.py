"""Overlap of copies and kernels in the LAST driver-pipeline call of a
rocprofv3 trace of tools/driver_pipeline_trace.py.

The call is the last `blobs` dispatches of `kernel`; its window runs from the
first host-to-device copy that ends after the previous call's last kernel to
the last device-to-host copy that starts before the window's end.  Reported:
the window, each engine's busy time (union of its intervals: uploads, kernels,
downloads), their sum over the window (how many of the three run at once on
average), and a lane chart per queue.

    python tools/trace_overlap.py OUT_DIR [kernel] [blobs]
"""
import csv
import glob
import os
import sys

root = sys.argv[1]
kernel = sys.argv[2] if len(sys.argv) > 2 else "lcg"
blobs = int(sys.argv[3]) if len(sys.argv) > 3 else 16


def rows(pattern):
    f = glob.glob(os.path.join(root, "**", pattern), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


allk = rows("*kernel_trace.csv")
ks = [r for r in allk if kernel in r["Kernel_Name"]]
ks.sort(key=lambda r: int(r["Start_Timestamp"]))
if len(ks) < 2 * blobs:
    raise SystemExit(f"only {len(ks)} '{kernel}' dispatches")
call, prev = ks[-blobs:], ks[-2 * blobs:-blobs]
t_prev = max(int(r["End_Timestamp"]) for r in prev)
k_end = max(int(r["End_Timestamp"]) for r in call)
cp = rows("*memory_copy_trace.csv")
dir_key = next((k for k in (cp[0].keys() if cp else []) if k.lower() in ("direction", "operation", "kind")), None)


def direction(r):
    v = (r.get("Direction") or r.get("Operation") or r.get("Kind") or "").upper()
    if "HOST_TO_DEVICE" in v or "H2D" in v:
        return "h2d"
    if "DEVICE_TO_HOST" in v or "D2H" in v:
        return "d2h"
    return "other"


ups = [r for r in cp if direction(r) == "h2d" and int(r["End_Timestamp"]) > t_prev and int(r["Start_Timestamp"]) < k_end]
downs = [r for r in cp if direction(r) == "d2h" and int(r["Start_Timestamp"]) > t_prev]
# ROCclr runs device-to-host copies into pinned memory as blit kernels
# (__amd_rocclr_copyBuffer) on a hardware queue: those count as downloads
downs += [r for r in allk if "copyBuffer" in r["Kernel_Name"] and int(r["Start_Timestamp"]) > t_prev]
# this call's downloads: after its first kernel ends (earlier ones finish the
# previous call's blobs), before 5 ms past its last kernel
k_first_end = min(int(r["End_Timestamp"]) for r in call)
downs = [r for r in downs if k_first_end <= int(r["Start_Timestamp"]) <= k_end + 5_000_000]
w0 = min([int(r["Start_Timestamp"]) for r in ups + call])
w1 = max([int(r["End_Timestamp"]) for r in downs + call])


def busy(rs):
    iv = sorted((max(w0, int(r["Start_Timestamp"])), min(w1, int(r["End_Timestamp"]))) for r in rs)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


win = w1 - w0
b = {"uploads": busy(ups), "kernels": busy(call), "downloads": busy(downs)}
print(f"# Driver pipeline, last call: {blobs} blobs of `{kernel}`\n")
print(f"window {win / 1e6:.3f} ms; busy: " + ", ".join(f"{k} {v / 1e6:.3f} ms" for k, v in b.items()) +
      f"; sum / window = **{sum(b.values()) / win:.2f}** (1.0 = nothing overlaps, 3.0 = all three always)\n")
print(f"copies in the window: {len(ups)} uploads, {len(downs)} downloads; kernels {len(call)}\n")
print("| # | what | queue / engine | start µs | end µs |")
print("|---|---|---|---|---|")
ev = [("H2D", r) for r in ups] + [("kernel", r) for r in call] + \
    [("D2H" + (" (blit kernel)" if "Kernel_Name" in r else ""), r) for r in downs]
ev.sort(key=lambda p: int(p[1]["Start_Timestamp"]))
for i, (what, r) in enumerate(ev):
    lane = ("queue " + r["Queue_Id"]) if r.get("Queue_Id") else ("SDMA, stream " + (r.get("Stream_Id") or "?"))
    print(f"| {i} | {what} | {lane} | {(int(r['Start_Timestamp']) - w0) / 1e3:.1f} | {(int(r['End_Timestamp']) - w0) / 1e3:.1f} |")
