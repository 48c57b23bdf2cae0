"""Where one pool consumer's host time per task goes (one whole GPU, tiny
device-resident tasks): the Python enqueue, the native issue (Cores::compute:
launch + marker), the marker polls, and the rest of the consumer loop.

    python tools/pool_cost_probe.py [tasks] > gpurun_out/pool_cost.json
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
TASKS = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
out = {}
for queues in (1, 3):
    pool = ClDevicePool(ClDevicePoolType.DEVICE_COMPUTE_AT_WILL, SRC, True, queues)
    pool.add_device(ck.ClPlatforms.all().gpus()[0])
    v = ck.ClArray(np.array([1.0], np.float32))
    v.write = False
    xs = [ck.ClArray(np.zeros(256, np.float32)) for _ in range(64)]
    for x in xs:
        x.read = x.write = False
        pool.crunchers[0].upload(x)
    pool.crunchers[0].upload(v)
    v.read = False

    def batch(k):
        t = ClTaskPool()
        for i in range(k):
            t.feed(xs[i % 64].next_param(v).task(3, "add", 256, 256))
        return t

    pool.enqueue_task_pool(batch(512))
    pool.finish()
    p0 = pool._native.host_profile()
    tp = batch(TASKS)
    t0 = time.perf_counter()
    pool.enqueue_task_pool(tp)
    t1 = time.perf_counter()
    pool.finish()
    t2 = time.perf_counter()
    p1 = pool._native.host_profile()
    d = [b - a for a, b in zip(p0, p1)]
    out[f"q{queues}"] = {"tasks_per_s": round(TASKS / (t2 - t0)),
                         "python_enqueue_us_per_task": round((t1 - t0) * 1e6 / TASKS, 3),
                         "issue_us_per_task": round(d[0] * 1e3 / max(1, d[2]), 3),
                         "poll_us_per_poll": round(d[1] * 1e3 / max(1, d[3]), 3),
                         "polls_per_task": round(d[3] / max(1, d[2]), 3),
                         "wall_us_per_task": round((t2 - t0) * 1e6 / TASKS, 3)}
    pool.dispose()
from cekirdekler_amd._native import cek  # noqa: E402
from cekirdekler_amd.ops.library import code_object  # noqa: E402

r = cek.launch_rate_probe(0, code_object("stream"), "cek_copy_u8", 1, 4000)
out["raw_hip_launch_us"] = round(1e3 * r["host_ms"] / 4000, 3)
print(json.dumps(out), flush=True)
