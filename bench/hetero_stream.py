"""CPU + GPU co-execution on host-resident data: the case the reference's
load balancer exists for (Cores.cs:130-135 shares, README "CPU+GPU" and
Kamera.cs:266's "3× as fast" claim), measured where it can pay.

Each compute reads two host arrays and writes one back — every call moves
its data over PCIe for the GPU, while the CPU device works on the same
pinned pages in place.  Per element the kernel runs ``iters`` dependent
FMAs, so the sweep moves from a streaming kernel (the GPU is bound by the
host link, the CPU by its memory bandwidth) to compute-heavier ones (the
CPU falls behind).  Configs, interleaved round by round so host-load drift
hits every config alike:

* ``cpu``      — the CPU device alone (its threads sized to the process's
  CPU share, ``hardware.usable_cpus``);
* ``gpu``      — the GPU alone, event pipeline (``pipeline_blobs`` chunks:
  upload, kernel and download of different chunks overlap);
* ``gpu+cpu``  — both, the reference balancing law splitting the range and
  the GPU's part pipelined the same way;
* ``gpu+cpu_fit`` — both, with the overhead-aware balancer (it fits
  t = a + b·range per device and may drop a device whose share does not pay
  for its fixed cost; here it should keep both).

``speedup_over_cpu`` / ``speedup_over_gpu`` per intensity are the headline;
``shares`` is where the balancer settled.  Results verified against numpy.
"""
import argparse
import statistics
import time

import numpy as np

from common import emit

import cekirdekler_amd as ck

SRC = """
__global__ void poly(const float* x, float* y) {
    long long i = get_global_id(0);
    float v = x[i], acc = y[i];
    for (int k = 0; k < ITERS; ++k) acc = fmaf(acc, v, 0.25f);
    y[i] = acc;
}
"""

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=64 << 20, help="elements per array (default 256 MiB each)")
ap.add_argument("--iters", default="1,16,64")
ap.add_argument("--calls", type=int, default=6, help="timed calls per round and config")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--warm", type=int, default=25, help="balancer convergence calls")
ap.add_argument("--blobs", type=int, default=8)
ap.add_argument("--order", default="",
                help="comma list of configs in run order (a name may repeat with a _N suffix: "
                     "gpu+cpu_2 is a second law cruncher); default cpu,gpu,gpu+cpu,gpu+cpu_fit")
ap.add_argument("--records", action="store_true",
                help="keep each mixed cruncher's per-call record (wall, per-device ms, GPU share)")
ap.add_argument("--cpu-threads", type=int, default=-1,
                help="cap on the CPU device's threads (default: the process's CPU share minus one)")
a = ap.parse_args()

plats = ck.ClPlatforms.all()
cpu, gpus = plats.cpus(True, max_cpu_cores=a.cpu_threads), plats.gpus()
n = a.n
rng = np.random.default_rng(0)
x = ck.ClArray(n, np.float32)
x.array[:] = rng.uniform(-0.9, 0.9, n).astype(np.float32)
x.read_only = True
x.partial_read = True
y = ck.ClArray(n, np.float32)
y0 = rng.uniform(-1.0, 1.0, n).astype(np.float32)
y.partial_read = True

configs = [("cpu", cpu)]
if len(gpus):
    configs += [("gpu", gpus[0]), ("gpu+cpu", gpus[0] + cpu), ("gpu+cpu_fit", gpus[0] + cpu)]
if a.order:
    base = {"cpu": lambda: cpu, "gpu": lambda: gpus[0], "gpu+cpu": lambda: gpus[0] + cpu,
            "gpu+cpu_fit": lambda: gpus[0] + cpu}
    configs = []
    for name in a.order.split(","):
        key = name if name in base else name.rsplit("_", 1)[0]
        configs.append((name, base[key]()))

out = {"config": "hetero_stream", "n": n, "bytes_per_call": 12 * n, "cpu_threads": cpu.device(0).native_info().cpu_threads,
       "timing": f"median of {a.rounds} interleaved rounds of {a.calls} calls per config",
       "pipeline_blobs": a.blobs, "devices": {}}


def expected(iters: int, idx: np.ndarray) -> np.ndarray:
    xv = x.array[idx].astype(np.float32)
    acc = y0[idx].astype(np.float32)
    for _ in range(iters):
        acc = (acc.astype(np.float64) * xv + 0.25).astype(np.float32)
    return acc


for iters in [int(s) for s in a.iters.split(",")]:
    src = SRC.replace("ITERS", str(iters))
    crs = {}
    for name, devs in configs:
        cr = ck.ClNumberCruncher(devs, src)
        if name.endswith("_fit"):  # the overhead-aware balancer (t = a + b·range per device)
            cr.overhead_aware_balancer = True
        out["devices"][name] = cr.device_names()
        crs[name] = cr

    def call(cr):
        x.next_param(y).compute(cr, 1, "poly", n, 256, pipeline=True, pipeline_blobs=a.blobs)

    for name, cr in crs.items():
        for _ in range(a.warm):
            call(cr)
    runs = {name: [] for name in crs}
    recs = {name: [] for name in crs if "+" in name}
    for _ in range(a.rounds):
        for name, cr in crs.items():
            t = time.perf_counter()
            for _ in range(a.calls):
                call(cr)
                if a.records and name in recs:
                    r = cr.last_record()
                    rr = r["ranges"]
                    recs[name].append([round(r["wall_ms"], 3), [round(v, 3) for v in r["device_ms"]],
                                       round(rr[0] / max(1, sum(rr)), 4)])
            runs[name].append((time.perf_counter() - t) * 1e3 / a.calls)
    res = {}
    probe = np.concatenate([np.arange(0, 4096), rng.integers(0, n, 4096), np.arange(n - 4096, n)])
    for name, cr in crs.items():
        y.array[:] = y0
        call(cr)
        got = y.array[probe]
        ref = expected(iters, probe)
        ms = statistics.median(runs[name])
        r = {"ms": ms, "ms_rounds": [round(v, 3) for v in runs[name]],
             "GBps": 12 * n / ms / 1e6, "gflops": 2 * iters * n / ms / 1e6,
             "max_abs_err": float(np.abs(got - ref).max())}
        if "+" in name:
            rr = cr.ranges(1)
            r["shares"] = [v / sum(rr) for v in rr]
        if a.records and name in recs:
            r["records"] = recs[name]
        if name.endswith("_fit"):
            r["predictor"] = cr.balancer_predictor_info(1)
        res[name] = r
        cr.dispose()
    if all(k in res for k in ("cpu", "gpu", "gpu+cpu")):
        res["speedup_over_cpu"] = res["cpu"]["ms"] / res["gpu+cpu"]["ms"]
        res["speedup_over_gpu"] = res["gpu"]["ms"] / res["gpu+cpu"]["ms"]
        res["ideal_ms"] = 1.0 / (1.0 / res["cpu"]["ms"] + 1.0 / res["gpu"]["ms"])
    out[f"iters_{iters}"] = res
emit(out)
