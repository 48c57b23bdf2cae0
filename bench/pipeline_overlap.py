"""The reference's host<->device pipelining claim on a BALANCED workload
(VERDICT r4 next #5).

``Cores.cs:467`` claims "up to 3x" for the read/compute/write pipeline when
read, compute and write each take about a third of a call.  This bench builds
exactly that case and runs it through ``compute()`` three ways:

* ``3phase``  — no pipeline: upload the device's whole range, run the kernel,
  download the result (Cores.cs:747-834);
* ``event``   — the event-driven pipeline (Cores.cs:1197-1367): two
  interleaved half-pipelines of {upload, kernel, download} streams with
  event edges, at 4 / 8 / 16 blobs;
* ``driver``  — the driver-driven pipeline (Cores.cs:1368-1958): blob k's
  kernels on queue k mod Q, at 4 / 8 / 16 blobs.  Default layout: the
  uploads in the main stream's one chain of copies, the downloads on one
  download stream, each gated by events (``_inqueue``: the reference's
  upload→kernel→download in order on the queue; ``_readsq``: uploads in the
  queue, downloads on their own stream).

The kernel is a user kernel string (hiprtc), one uint32 in and one out per
work item, with ``iters`` LCG steps per element.  ``iters`` is calibrated at
start so the kernel alone takes as long as the mean of the upload and the
download (the upload timed alone through ``compute()``, the download as the
difference of upload + download and upload alone).  Every timed call's output is checked EXACTLY
against the closed form of the iterated LCG (``v -> a^n v + c(a^n-1)/(a-1)``
mod 2^32), so no mode can skip work.

Stream-topology A/B: the event pipeline's default
layout (uploads on the main stream, two kernel and two download streams = 5
streams) against a 4-stream layout (one download stream), and the driver
pipeline on Q = 4 queues (the hardware queue count, the default) against
Q = 16 (the reference's fixed count).  Configs are interleaved round by
round; each reports the median.
"""
import argparse
import statistics
import time

import numpy as np

from common import emit, sync

import cekirdekler_amd as ck

A_LCG, C_LCG = 1664525, 1013904223

SRC = """
__global__ void lcg(const unsigned int* x, const int* it, unsigned int* y) {
    long long i = get_global_id(0);
    unsigned int v = x[i];
    const int n = it[0];
    for (int k = 0; k < n; ++k) v = v * 1664525u + 1013904223u;
    y[i] = v;
}
"""


def lcg_power(n: int):
    """(A, C) with f^n(v) = A v + C (mod 2^32) for f(v) = a v + c."""
    A, C = 1, 0  # identity
    pa, pc = A_LCG, C_LCG  # f^(2^k)
    while n:
        if n & 1:
            A, C = (pa * A) & 0xFFFFFFFF, (pa * C + pc) & 0xFFFFFFFF
        pa, pc = (pa * pa) & 0xFFFFFFFF, (pa * pc + pc) & 0xFFFFFFFF
        n >>= 1
    return A, C


def expected(x: np.ndarray, n: int) -> np.ndarray:
    A, C = lcg_power(n)
    return ((x.astype(np.uint64) * np.uint64(A) + np.uint64(C)) & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=64 << 20, help="uint32 elements (default 256 MiB in + 256 MiB out)")
    ap.add_argument("--blobs", default="4,8,16")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--calls", type=int, default=3, help="timed calls per round and config")
    ap.add_argument("--device", choices=("gpu", "cpu"), default="gpu")
    ap.add_argument("--iters", type=int, default=0, help="LCG steps per element (0: calibrate)")
    a = ap.parse_args()

    plats = ck.ClPlatforms.all()
    dev = plats.gpus()[0] if a.device == "gpu" else plats.cpus(True)
    n, L = a.n, 256
    blobs = [int(b) for b in a.blobs.split(",") if b]
    rng = np.random.default_rng(0)
    x = ck.ClArray(n, np.uint32)
    x.array[:] = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
    x.partial_read = True
    x.write = False
    it = ck.ClArray(np.zeros(1, np.int32))
    it.write = False
    y = ck.ClArray(n, np.uint32)
    y.read = False

    # the default compute-stream count (hardware queues minus the main
    # stream's, hardware.async_queue_count), one per hardware queue (4) and
    # the reference's 16
    crs = {"qd": ck.ClNumberCruncher(dev, SRC), "q4": ck.ClNumberCruncher(dev, SRC, queue_concurrency=4),
           "q16": ck.ClNumberCruncher(dev, SRC, queue_concurrency=16)}
    for cr in crs.values():
        if cr.error_code():
            raise SystemExit(cr.error_message())
    cr = crs["qd"]
    qd = cr.compute_queue_concurrency
    cid = iter(range(1, 1000))

    def call(c, compute_id, pipeline=False, ptype=ck.PIPELINE_EVENT, nb=1):
        x.next_param(it, y).compute(c, compute_id, "lcg", n, L, 0, pipeline, ptype, nb)

    def med_ms(fn, calls):
        sync()
        t = time.perf_counter()
        for _ in range(calls):
            fn()
        sync()
        return (time.perf_counter() - t) * 1e3 / calls

    # ---- calibration: upload alone, upload + download, kernel per LCG step ----
    # (the download's share is the difference of the first two, both through
    # the same 3-phase path the baseline config runs)
    id_up, id_down, id_k = next(cid), next(cid), next(cid)
    it.array[0] = 0
    y.write = False
    call(cr, id_up)  # first upload also creates the buffers
    up_ms = statistics.median(med_ms(lambda: call(cr, id_up), 3) for _ in range(3))
    y.write = True
    call(cr, id_down)
    both_ms = statistics.median(med_ms(lambda: call(cr, id_down), 3) for _ in range(3))
    down_ms = max(0.0, both_ms - up_ms)
    x.read = x.partial_read = False  # x stays on the device (a partial read uploads whatever .read says)
    y.write = False
    probe = 256
    it.array[0] = probe
    call(cr, id_k)
    k_probe_ms = statistics.median(med_ms(lambda: call(cr, id_k), 3) for _ in range(3))
    it.array[0] = 0
    zero_ms = statistics.median(med_ms(lambda: call(cr, id_k), 3) for _ in range(3))
    per_step = max(1e-9, (k_probe_ms - zero_ms) / probe)
    iters = a.iters or max(1, int(round(((up_ms + down_ms) / 2 - zero_ms) / per_step)))
    it.array[0] = iters
    kernel_ms = statistics.median(med_ms(lambda: call(cr, id_k), 3) for _ in range(3))
    x.read = x.partial_read = True
    y.write = True
    want = expected(x.array, iters)

    # ---- configs --------------------------------------------------------------
    configs = [("3phase", lambda c, i: call(crs["qd"], i), None)]
    for b in blobs:
        configs.append((f"event_b{b}", lambda c, i, b=b: call(crs["qd"], i, True, ck.PIPELINE_EVENT, b), None))
        configs.append((f"event_b{b}_4streams", lambda c, i, b=b: call(crs["q16"], i, True, ck.PIPELINE_EVENT, b),
                        "writes_one_stream"))
        configs.append((f"driver_b{b}_qd", lambda c, i, b=b: call(crs["qd"], i, True, ck.PIPELINE_DRIVER, b), None))
        configs.append((f"driver_b{b}_q4", lambda c, i, b=b: call(crs["q4"], i, True, ck.PIPELINE_DRIVER, b), None))
        configs.append((f"driver_b{b}_q16", lambda c, i, b=b: call(crs["q16"], i, True, ck.PIPELINE_DRIVER, b), None))
        # the reference's layout: each blob's upload, kernels and download in
        # order on its queue (driver_reads_on_main_stream and
        # driver_downloads_own_stream off); and uploads in the queue with the
        # downloads on their own stream
        configs.append((f"driver_b{b}_inqueue", lambda c, i, b=b: call(crs["qd"], i, True, ck.PIPELINE_DRIVER, b),
                        "downloads_in_queue"))
        configs.append((f"driver_b{b}_readsq", lambda c, i, b=b: call(crs["qd"], i, True, ck.PIPELINE_DRIVER, b),
                        "reads_in_queue"))
    ids = {name: next(cid) for name, _, _ in configs}
    times = {name: [] for name, _, _ in configs}
    exact = {name: True for name, _, _ in configs}
    piped, moved = {}, {}

    def run(name, fn, layout):
        if layout in ("reads_in_queue", "downloads_in_queue"):
            cc = crs["qd"].cores
            cc.driver_reads_on_main_stream = False
            cc.driver_downloads_own_stream = layout == "reads_in_queue"
            try:
                return fn(None, ids[name])
            finally:
                cc.driver_reads_on_main_stream = True
                cc.driver_downloads_own_stream = True
        c = crs["q16"] if layout else None
        if c is not None:
            c.cores.pipeline_writes_one_stream = True
        try:
            return fn(None, ids[name])
        finally:
            if c is not None:
                c.cores.pipeline_writes_one_stream = False

    for name, fn, layout in configs:  # untimed: buffers, balancer state, streams
        y.array[:] = 0
        run(name, fn, layout)
        exact[name] &= bool(np.array_equal(y.array, want))
        c = crs["q16"] if ("q16" in name or layout == "writes_one_stream") else (
            crs["q4"] if name.endswith("_q4") else crs["qd"])
        rec = c.last_record()
        piped[name] = bool(rec["pipelined"])
        moved[name] = [int(rec["h2d_bytes"]), int(rec["d2h_bytes"])]
    for _ in range(a.rounds):
        for name, fn, layout in configs:
            y.array[:] = 0
            times[name].append(med_ms(lambda: run(name, fn, layout), a.calls))
            exact[name] &= bool(np.array_equal(y.array, want))
    res = {name: round(statistics.median(v), 3) for name, v in times.items()}
    base = res["3phase"]
    ev = min((k for k in res if k.startswith("event_") and not k.endswith("4streams")), key=res.get)
    ev4 = min((k for k in res if k.endswith("4streams")), key=res.get)
    dqd = min((k for k in res if k.startswith("driver_") and k.endswith("_qd")), key=res.get)
    dq4 = min((k for k in res if k.startswith("driver_") and k.endswith("_q4")), key=res.get)
    dq16 = min((k for k in res if k.endswith("q16")), key=res.get)
    dinq = min((k for k in res if k.endswith("_inqueue")), key=res.get)
    drq = min((k for k in res if k.endswith("_readsq")), key=res.get)
    parts = [up_ms, kernel_ms, down_ms]
    out = {
        "config": "pipeline_overlap_balanced",
        "n": n, "bytes_per_call": 8 * n, "lcg_iters": iters,
        "read_compute_write_ms": [round(v, 3) for v in parts],
        "ideal_speedup_sum_over_max": round(sum(parts) / max(parts), 3),
        "ms": res,
        "pipelined": piped,
        # H2D / D2H bytes of one call per config: every config moves the same data
        "same_bytes_every_config": len({tuple(v) for v in moved.values()}) == 1,
        "h2d_d2h_bytes_per_call": moved.get("3phase"),
        "outputs_exact": all(exact.values()),
        "default_compute_streams": qd,
        "best_event": ev, "best_event_4streams": ev4, "best_driver_default": dqd, "best_driver_q4": dq4,
        "best_driver_q16": dq16,
        "pipeline_speedup_event": round(base / min(res[ev], res[ev4]), 3),
        "pipeline_speedup_driver": round(base / min(res[dqd], res[dq4], res[dq16]), 3),
        "pipeline_speedup_driver_in_queue": round(base / res[dinq], 3),
        "event_5_vs_4_streams": [res[ev], res[ev4]],
        "driver_default_q4_q16": [res[dqd], res[dq4], res[dq16]],
        "best_driver_downloads_in_queue": dinq,
        "driver_own_download_stream_vs_in_queue": [res[dqd], res[dinq]],
        "best_driver_reads_in_queue": drq,
        "pipeline_speedup_driver_reads_in_queue": round(base / res[drq], 3),
        "timing": f"median of {a.rounds} interleaved rounds of {a.calls} calls per config",
    }
    for c in crs.values():
        c.dispose()
    emit(out)


if __name__ == "__main__":
    main()
