"""GPU probe for the reference's fine-grained queue control claim
(kernel-to-kernel gap 2-3 µs → 150-300 µs with markers,
ClNumberCruncher.cs:79 / Cores.cs:447).  Runs 400 back-to-back tiny computes
in enqueue mode, once with fine_grained_queue_control off (kernel k_off) and
once on (k_on: a hipStreamWriteValue64 marker after every compute).  Run
under ``rocprofv3 --kernel-trace`` and read the gaps with
``tools/marker_gap_probe.py --analyze <db>``."""
import os
import sqlite3
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def analyze(db: str) -> None:
    import statistics

    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end from kernels order by start"))
    for name in ("k_off", "k_on"):
        ks = [(s, e) for n, s, e in rows if n == name]
        gaps = [(ks[i + 1][0] - ks[i][1]) / 1e3 for i in range(len(ks) - 1)]
        gaps = gaps[20:]  # warm-up
        print(f"{name}: {len(ks)} dispatches, end→start gap µs: median {statistics.median(gaps):.2f}, "
              f"p90 {sorted(gaps)[int(0.9 * len(gaps))]:.2f}, "
              f"kernel µs median {statistics.median([(e - s) / 1e3 for s, e in ks]):.2f}")


def run() -> None:
    import numpy as np

    import cekirdekler_amd as ck

    src = """__global__ void k_off(float* x) { x[get_global_id(0)] += 1.0f; }
             __global__ void k_on(float* x) { x[get_global_id(0)] += 1.0f; }"""
    cr = ck.ClNumberCruncher(ck.ClPlatforms.all().gpus()[0], src)
    x = ck.ClArray(1 << 14, np.float32)
    x.read = x.write = False
    for name, fine in (("k_off", False), ("k_on", True)):
        cr.fine_grained_queue_control = fine
        x.compute(cr, 1, name, 1 << 14, 256)
        cr.enqueue_mode = True
        t = time.perf_counter()
        for _ in range(400):
            x.compute(cr, 1, name, 1 << 14, 256)
        host = (time.perf_counter() - t) * 1e6 / 400
        cr.enqueue_mode = False
        print(f"{name}: host µs per compute {host:.1f}, markers reached {cr.count_markers_reached()}")
    cr.dispose()


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    else:
        run()
