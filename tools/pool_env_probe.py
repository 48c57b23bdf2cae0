"""Why one pool consumer dispatches slower inside bench/task_pool.py than in
a fresh process (tools/pool_cost_probe.py): the same one-device dispatch
measured (a) fresh, (b) with the library code objects the bench's pool
loads, (c) with a CU-partitioned cruncher alive in the process, (d) both.

    python tools/pool_env_probe.py > gpurun_out/pool_env.json
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.ops.library import library  # noqa: E402
from cekirdekler_amd.parallel.pool import ClDevicePool, ClDevicePoolType, ClTaskPool  # noqa: E402

SRC = """__global__ void add(float* x, const float* v) { long long i = get_global_id(0); x[i] = x[i] * 2.0f + v[0]; }"""
TASKS = 4096
g = ck.ClPlatforms.all().gpus()


def rate(prebuilt=None, queues=1, devices=None):
    pool = ClDevicePool(ClDevicePoolType.DEVICE_COMPUTE_AT_WILL, SRC, True, queues, prebuilt=prebuilt)
    pool.add_device(g[0] if devices is None else devices)
    v = ck.ClArray(np.array([1.0], np.float32))
    v.write = False
    xs = [ck.ClArray(np.zeros(256, np.float32)) for _ in range(64)]
    for x in xs:
        x.read = x.write = False
        for cr in pool.crunchers:
            cr.upload(x)
    for cr in pool.crunchers:
        cr.upload(v)
    v.read = False

    def batch(k):
        t = ClTaskPool()
        for i in range(k):
            t.feed(xs[i % 64].next_param(v).task(3, "add", 256, 256))
        return t

    pool.enqueue_task_pool(batch(512))
    pool.finish()
    best = 0
    for _ in range(3):
        tp = batch(TASKS)
        t0 = time.perf_counter()
        pool.enqueue_task_pool(tp)
        pool.finish()
        best = max(best, TASKS / (time.perf_counter() - t0))
    prof = pool._native.host_profile()
    pool.dispose()
    return {"tasks_per_s": round(best), "issue_us_per_task": round(prof[0] * 1e3 / max(1, prof[2]), 3)}


LIBS = library("sgemm_bf16", "reduce", "nbody", "mandelbrot", "stream")
if len(sys.argv) > 1:
    # one case per process, for a HIP API trace of each (rocprofv3 --hip-trace --stats):
    # "fresh" = one queue in a fresh process; "after_q3" = the same after a
    # 3-queue pool has come and gone
    case = sys.argv[1]
    if case == "after_q3":
        rate(queues=3)
    devices = None
    if case == "parts8":  # 8 CU partitions, one stream each (the bench's pool)
        devices = g[0:1].cu_partitions(8)
    elif case == "logical8":  # 8 whole-GPU logical devices, one stream each
        devices = g[0]
        for _ in range(7):
            devices = devices + g[0]
    print(json.dumps({case: rate(prebuilt=LIBS if case.endswith("_libs") else None, devices=devices)}),
          flush=True)
    sys.exit(0)
out = {"fresh": rate(), "fresh_q3": rate(queues=3), "libs": rate(LIBS)}
def touch(cr):  # one compute: the cruncher's streams exist
    x = ck.ClArray(np.zeros(256, np.float32))
    v = ck.ClArray(np.ones(256, np.float32))
    x.next_param(v).compute(cr, 1, "add", 256, 256)


part = ck.ClNumberCruncher(g[0:1].cu_partitions(8)[0], SRC)
touch(part)
out["with_partition_cruncher"] = rate()
out["with_partition_cruncher_libs"] = rate(LIBS)
cp = g[0:1].cu_partitions(8)
parts = [ck.ClNumberCruncher(cp[i], SRC, queue_concurrency=1) for i in range(len(cp))]
for c in parts:
    touch(c)
out["with_8_partition_crunchers"] = rate()
for c in parts:
    c.dispose()
part.dispose()
out["after_dispose"] = rate()
print(json.dumps(out), flush=True)
