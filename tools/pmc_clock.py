"""Per-kernel clock and matrix-core use from a rocprofv3 run with
``--pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace``:
GHz = GRBM_GUI_ACTIVE / 8 XCDs / duration; MFMA use per cycle =
SQ_VALU_MFMA_BUSY_CYCLES × 1024 FLOP / (cycles × 256 CUs × 4069 FLOP/clk)
(the 16x16x32 bf16 rate; 1024 FLOP per busy unit measured on mfma_peak).

    python tools/pmc_clock.py <output dir> [kernel substring]
"""
import collections
import csv
import glob
import os
import statistics
import sys

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
disp = collections.defaultdict(dict)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
            continue
        d = disp[(r["Kernel_Name"], r["Correlation_Id"])]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d["dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
by_kernel = collections.defaultdict(list)
for (k, _), d in disp.items():
    if d.get("dur_ns") and "GRBM_GUI_ACTIVE" in d:
        cyc = d["GRBM_GUI_ACTIVE"] / 8
        use = d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) * 1024 / (cyc * 256 * 4069)
        by_kernel[k].append((d["dur_ns"] / 1e3, cyc / d["dur_ns"], use))
for k, v in by_kernel.items():
    v = v[len(v) // 3:]  # drop the clock ramp of the first third
    print(f"| `{k[:50]}` | {len(v)} | {statistics.median(x[0] for x in v):.1f} | "
          f"{statistics.median(x[1] for x in v):.3f} | {100 * statistics.median(x[2] for x in v):.1f} |")
