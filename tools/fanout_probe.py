"""Host cost of one compute() against the number of logical devices (1, 2,
4, 8 copies of GPU 0): enqueue mode, sync mode and graph replay, tiny
kernels (4096 work items per device); plus DevicePool dispatch throughput
with near-zero-cost tasks at 1/2/4/8 consumers for both device policies.
Run it under CEK_SPIN_US=0 and the default to compare the worker hand-off.

    python tools/fanout_probe.py [out.json]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.parallel.pool import ClDevicePool, ClDevicePoolType, ClTaskPool  # noqa: E402

SRC = "__global__ void inc(float* x) { x[get_global_id(0)] += 1.0f; }"


def per_compute(ndev, reps=2000):
    g0 = ck.ClPlatforms.all().gpus()[0]
    devs = g0
    for _ in range(ndev - 1):
        devs = devs + g0
    cr = ck.ClNumberCruncher(devs, SRC)
    n = 4096 * ndev
    x = ck.ClArray(np.zeros(n, np.float32))
    x.compute(cr, 1, "inc", n, 256)
    x.read = x.write = False
    for _ in range(50):
        x.compute(cr, 1, "inc", n, 256)
    out = {}
    cr.enqueue_mode = True
    for _ in range(100):
        x.compute(cr, 1, "inc", n, 256)
    cr.enqueue_mode = False
    cr.enqueue_mode = True
    t = time.perf_counter()
    for _ in range(reps):
        x.compute(cr, 1, "inc", n, 256)
    host = (time.perf_counter() - t) * 1e6 / reps
    cr.enqueue_mode = False
    total = (time.perf_counter() - t) * 1e6 / reps
    out["enqueue_host_us"] = round(host, 2)
    out["enqueue_total_us"] = round(total, 2)
    t = time.perf_counter()
    for _ in range(reps // 4):
        x.compute(cr, 1, "inc", n, 256)
    out["sync_us"] = round((time.perf_counter() - t) * 1e6 / (reps // 4), 2)
    with cr.capture() as g:
        for _ in range(100):
            x.compute(cr, 1, "inc", n, 256)
    g.replay(3)
    t = time.perf_counter()
    g.replay(20)
    out["graph_us"] = round((time.perf_counter() - t) * 1e6 / 2000, 2)
    g.destroy()
    # build-only cost (Python side: flags -> native call description)
    grp = ck.ClParameterGroup([x])
    t = time.perf_counter()
    for _ in range(reps):
        cr._build_call(grp, 1, "inc", n, 256)
    out["python_build_call_us"] = round((time.perf_counter() - t) * 1e6 / reps, 2)
    cr.dispose()
    return out


def pool_rate(ndev, policy, tasks=4096, queues=4):
    g0 = ck.ClPlatforms.all().gpus()[0]
    devs = g0
    for _ in range(ndev - 1):
        devs = devs + g0
    pool = ClDevicePool(policy, SRC, True, queues)
    pool.add_device(devs)
    xs = [ck.ClArray(np.zeros(256, np.float32)) for _ in range(64)]
    for x in xs:
        x.read = x.write = False

    def run(k):
        tp = ClTaskPool()
        for i in range(k):
            tp.feed(xs[i % len(xs)].task(1, "inc", 256, 256))
        t = time.perf_counter()
        pool.enqueue_task_pool(tp)
        pool.finish()
        return time.perf_counter() - t

    run(256)
    dt = run(tasks)
    counts = pool.device_task_counts()
    pool.dispose()
    return {"tasks_per_s": round(tasks / dt), "ms": round(dt * 1e3, 2), "per_device": counts}


def main():
    res = {"spin_us": float(os.environ.get("CEK_SPIN_US", "50"))}
    for ndev in (1, 2, 4, 8):
        res[f"compute_{ndev}dev"] = per_compute(ndev)
        print(ndev, res[f"compute_{ndev}dev"], flush=True)
    for pol in (ClDevicePoolType.DEVICE_COMPUTE_AT_WILL, ClDevicePoolType.DEVICE_ROUND_ROBIN):
        for ndev in (1, 8):
            res[f"pool_{pol.name}_{ndev}"] = pool_rate(ndev, pol)
            print(pol.name, ndev, res[f"pool_{pol.name}_{ndev}"], flush=True)
    js = json.dumps(res)
    print(js)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            f.write(js + "\n")


if __name__ == "__main__":
    main()
