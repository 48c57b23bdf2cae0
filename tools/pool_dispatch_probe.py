"""Where the device pool's host time per task goes.

Three measurements on GPU 0:

* ``hip_launch_threads``: raw HIP launch rate from T native threads, each on
  its own stream of the one device (``cek.launch_rate_probe``: no runtime,
  no pool, no sync) — the ceiling any fan-out over logical devices of one
  GPU can reach;
* ``fanout_us_per_compute``: host µs per enqueue-mode compute() of one
  cruncher over D logical devices (worker hand-off + D launches);
* ``pool``: ClDevicePool dispatch rate on tiny tasks (one 256-thread
  work-group each) for D logical devices, whole-GPU or CU-partitioned, with
  1 or 3 queues per device.

    python tools/pool_dispatch_probe.py > gpurun_out/pool_dispatch.json
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.parallel.pool import ClDevicePool, ClDevicePoolType, ClTaskPool  # noqa: E402

SRC = """__global__ void add(float* x, const float* v) { long long i = get_global_id(0); x[i] = x[i] * 2.0f + v[0]; }"""
TASKS = 4096


def devices(d, part):
    g = ck.ClPlatforms.all().gpus()
    if part and d > 1:
        return g[0:1].cu_partitions(d)
    out = g[0]
    for _ in range(d - 1):
        out = out + g[0]
    return out


def pool_rate(d, part, queues):
    pool = ClDevicePool(ClDevicePoolType.DEVICE_COMPUTE_AT_WILL, SRC, True, queues)
    pool.add_device(devices(d, part))
    v = ck.ClArray(np.array([1.0], np.float32))
    v.write = False
    xs = [ck.ClArray(np.zeros(256, np.float32)) for _ in range(64)]
    for x in xs:
        x.read = x.write = False
    for cr in pool.crunchers:
        cr.upload(v)
        for x in xs:
            cr.upload(x)
    v.read = False

    def batch(k):
        t = ClTaskPool()
        for i in range(k):
            t.feed(xs[i % 64].next_param(v).task(3, "add", 256, 256))
        return t

    pool.enqueue_task_pool(batch(512))
    pool.finish()
    tp = batch(TASKS)
    t0 = time.perf_counter()
    pool.enqueue_task_pool(tp)
    pool.finish()
    rate = TASKS / (time.perf_counter() - t0)
    pool.dispose()
    return round(rate)


def fanout_us(d, calls=400, spans=True):
    """One cruncher over D logical devices of GPU 0, enqueue mode: host µs
    per compute() of a tiny kernel split over the D devices (the runtime's
    worker hand-off plus D launches).  Logical devices of one GPU record a
    begin/end event pair per compute and device (``spans``); distinct GPUs
    record one span per enqueued batch, so ``spans=False`` is their case."""
    cr = ck.ClNumberCruncher(devices(d, 0), SRC)
    cr.cores.device_spans = spans
    v = ck.ClArray(np.array([1.0], np.float32))
    x = ck.ClArray(np.zeros(256 * d, np.float32))
    v.write = False
    x.write = False
    x.next_param(v).compute(cr, 1, "add", 256 * d, 256)
    v.read = x.read = False
    cr.enqueue_mode = True
    for _ in range(50):
        x.next_param(v).compute(cr, 1, "add", 256 * d, 256)
    cr.enqueue_mode = False
    cr.enqueue_mode = True
    t0 = time.perf_counter()
    for _ in range(calls):
        x.next_param(v).compute(cr, 1, "add", 256 * d, 256)
    host = (time.perf_counter() - t0) * 1e6 / calls
    cr.enqueue_mode = False
    cr.dispose()
    return round(host, 2)


from cekirdekler_amd._native import cek  # noqa: E402
from cekirdekler_amd.ops.library import code_object  # noqa: E402

out = {"tasks": TASKS, "pool": {}, "hip_launch_threads": {}, "fanout_us_per_compute": {}}
for t in (1, 2, 4, 8):
    r = cek.launch_rate_probe(0, code_object("stream"), "cek_copy_u8", t, 4000)
    out["hip_launch_threads"][f"t{t}"] = {"launches_per_s": round(r["launches_per_s"]),
                                          "us_per_launch_per_thread": round(1e3 * r["host_ms"] / 4000, 3)}
for d in (1, 2, 4, 8):
    out["fanout_us_per_compute"][f"d{d}"] = fanout_us(d)
    out["fanout_us_per_compute"][f"d{d}_no_spans"] = fanout_us(d, spans=False)
for d in (1, 2, 4, 8):
    for part in (0, 1):
        if d == 1 and part:
            continue
        for q in (1, 3):
            out["pool"][f"d{d}_part{part}_q{q}"] = pool_rate(d, part, q)
print(json.dumps(out), flush=True)
