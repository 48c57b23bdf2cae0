"""GPU probe: a launch-bound loop of tiny computes (4096 work items each),
per compute: host-issued in enqueue mode vs replayed from a captured
compute graph (ClNumberCruncher.capture)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402

SRC = "__global__ void inc(float* x) { x[get_global_id(0)] += 1.0f; }"
out = {}
for ndev in (1, 2):
    g0 = ck.ClPlatforms.all().gpus()[0]
    devs = g0 if ndev == 1 else g0 + g0
    cr = ck.ClNumberCruncher(devs, SRC)
    n = 4096 * ndev
    x = ck.ClArray(np.zeros(n, np.float32))
    x.compute(cr, 1, "inc", n, 256)
    x.read = x.write = False
    with cr.capture() as g:
        for _ in range(100):
            x.compute(cr, 1, "inc", n, 256)
    g.replay(3)
    t = time.perf_counter()
    g.replay(20)
    graph = (time.perf_counter() - t) * 1e6 / 2000
    for _ in range(100):
        x.compute(cr, 1, "inc", n, 256)
    cr.enqueue_mode = True
    t = time.perf_counter()
    for _ in range(2000):
        x.compute(cr, 1, "inc", n, 256)
    cr.enqueue_mode = False
    enq = (time.perf_counter() - t) * 1e6 / 2000
    t = time.perf_counter()
    for _ in range(500):
        x.compute(cr, 1, "inc", n, 256)
    sync = (time.perf_counter() - t) * 1e6 / 500
    out[f"{ndev}_device"] = {"graph_us_per_compute": round(graph, 2), "enqueue_us_per_compute": round(enq, 2),
                             "sync_us_per_compute": round(sync, 2)}
    g.destroy()
    cr.dispose()
print(json.dumps(out), flush=True)
