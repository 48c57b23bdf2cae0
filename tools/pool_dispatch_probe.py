"""Where the device pool's host time per task goes.

Dispatch rate of ClDevicePool on tiny tasks (one 256-thread work-group
each), for D logical devices of GPU 0, whole-GPU or CU-partitioned, with 1
or 3 queues per device.  Then the raw launch rate of the same kernel from D
host threads, each on its own cruncher in enqueue mode (no pool, no markers):
if that rate also falls as D grows on one GPU, the cost is the HIP runtime
serialising launches to one device, not the pool's hand-off.

    python tools/pool_dispatch_probe.py > gpurun_out/pool_dispatch.json
"""
import json
import os
import sys
import threading
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


def raw_rate(d, part):
    """D host threads, each launching TASKS/D computes on its own
    single-device cruncher in enqueue mode (one drain at the end)."""
    devs = devices(d, part)
    crs = [ck.ClNumberCruncher(devs[i], SRC, queue_concurrency=1) for i in range(d)]
    v = ck.ClArray(np.array([1.0], np.float32))
    v.write = False
    xs = [ck.ClArray(np.zeros(256, np.float32)) for _ in range(d)]
    for i, cr in enumerate(crs):
        xs[i].read = xs[i].write = False
        cr.upload(v)
        cr.upload(xs[i])
    v.read = False
    for i, cr in enumerate(crs):
        xs[i].next_param(v).compute(cr, 1, "add", 256, 256)
    per = TASKS // d
    barrier = threading.Barrier(d + 1)

    def run(i):
        cr, x = crs[i], xs[i]
        barrier.wait()
        cr.enqueue_mode = True
        for _ in range(per):
            x.next_param(v).compute(cr, 1, "add", 256, 256)
        cr.enqueue_mode = False

    th = [threading.Thread(target=run, args=(i,)) for i in range(d)]
    for t in th:
        t.start()
    barrier.wait()
    t0 = time.perf_counter()
    for t in th:
        t.join()
    rate = per * d / (time.perf_counter() - t0)
    for cr in crs:
        cr.dispose()
    return round(rate)


out = {"tasks": TASKS, "pool": {}, "raw_threads": {}}
for d in (1, 2, 4, 8):
    for part in (0, 1):
        if d == 1 and part:
            continue
        for q in (1, 3):
            out["pool"][f"d{d}_part{part}_q{q}"] = pool_rate(d, part, q)
        out["raw_threads"][f"d{d}_part{part}"] = raw_rate(d, part)
print(json.dumps(out), flush=True)
