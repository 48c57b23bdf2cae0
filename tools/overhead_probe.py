"""GPU probe: host time per compute() for a tiny kernel, by transfer kind
and mode (enqueue mode = no host sync per call)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402

N = 1 << 14
src = "__global__ void k(const float* x, float* y) { long long i = get_global_id(0); y[i] = x[i] + 1.0f; }"
gpu = ck.ClPlatforms.all().gpus()
cr = ck.ClNumberCruncher(gpu[0], src)
out = {}
for pinned in (True, False):
    for kind in ("none", "h2d", "d2h", "both"):
        for enq in (False, True):
            x = ck.ClArray(N, np.float32) if pinned else ck.ClArray(np.zeros(N, np.float32))
            y = ck.ClArray(N, np.float32) if pinned else ck.ClArray(np.zeros(N, np.float32))
            x.read = kind in ("h2d", "both")
            x.write = False
            y.read = False
            y.write = kind in ("d2h", "both")
            g = x.next_param(y)
            for _ in range(20):
                g.compute(cr, 5, "k", N, 256)
            cr.enqueue_mode = enq
            t = time.perf_counter()
            for _ in range(200):
                g.compute(cr, 5, "k", N, 256)
            host = (time.perf_counter() - t) * 1e3 / 200
            cr.enqueue_mode = False
            total = (time.perf_counter() - t) * 1e3 / 200
            out[f"{'pinned' if pinned else 'pageable'}/{kind}/{'enqueue' if enq else 'sync'}"] = {
                "host_us_per_call": round(1e3 * host, 1), "total_us_per_call": round(1e3 * total, 1)}
            x.dispose()
            y.dispose()
print(json.dumps(out, indent=1))
cr.dispose()
