#!/usr/bin/env python3
"""Per-compute() host overhead on one GPU: a trivial kernel over resident
arrays (no transfers), timed at three layers — torch launch+sync (floor),
the native Cores::compute with a prebuilt ComputeCall, and the public
ClArray.compute() path.  Prints one JSON line per layer."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd import cek  # noqa: E402

SRC = "__global__ void inc(float* x) { x[get_global_id(0)] += 1.0f; }"
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
ITERS = 2000


def bench(fn, iters=ITERS):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


x_t = torch.zeros(N, device="cuda")


def torch_step():
    x_t.add_(1.0)
    torch.cuda.synchronize()


print(json.dumps({"layer": "torch add_+synchronize", "us": round(bench(torch_step), 2)}))

for devs_name in ("gpu0", "gpu0+gpu0"):
    g = ck.ClPlatforms.all().gpus()
    devs = g[0] if devs_name == "gpu0" else g[0] + g[0]
    cr = ck.ClNumberCruncher(devs, SRC)
    x = ck.ClArray(np.zeros(N, np.float32))
    x.compute(cr, 1, "inc", N, 256)
    x.read = False
    x.write = False
    call = cek.ComputeCall()
    call.kernels = ["inc"]
    call.arrays = [x._spec()]
    call.global_range = N
    call.local_range = 256
    call.compute_id = 1
    us_native = bench(lambda: cr._cores.compute(call))
    us_api = bench(lambda: x.compute(cr, 1, "inc", N, 256))
    rec = cr.last_record()
    print(json.dumps({"layer": "native Cores.compute", "devices": devs_name, "us": round(us_native, 2)}))
    print(json.dumps({"layer": "ClArray.compute", "devices": devs_name, "us": round(us_api, 2),
                      "wall_ms_record": rec["wall_ms"], "device_ms": rec["device_ms"]}))
    cr.dispose()
