"""CPU + GPU on one kernel over host-resident arrays: the load balancer
splits the range between the devices on every call of a compute id
(reference ``Cores.cs`` balancing law), the GPU's share streams over PCIe
through the event pipeline and the CPU device works on the same pages in
place.  Without a GPU the example runs on two CPU devices.

    python examples/cpu_gpu_coexecution.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402

SRC = """
__global__ void poly(const float* x, float* y) {
    long long i = get_global_id(0);
    float v = x[i], acc = y[i];
    for (int k = 0; k < 16; ++k) acc = fmaf(acc, v, 0.25f);
    y[i] = acc;
}
"""

plats = ck.ClPlatforms.all()
cpu = plats.cpus(True)
devices = (plats.gpus()[0] + cpu) if len(plats.gpus()) else (cpu + cpu)
cr = ck.ClNumberCruncher(devices, SRC)

n = 1 << 24
x = ck.ClArray(n, np.float32)  # pinned host memory
x.array[:] = np.random.default_rng(0).uniform(-0.9, 0.9, n).astype(np.float32)
x.read_only = True
x.partial_read = True  # each device reads only its own slice
y = ck.ClArray(n, np.float32)
y.partial_read = True

for call in range(12):
    t = time.perf_counter()
    x.next_param(y).compute(cr, 1, "poly", n, 256, pipeline=True, pipeline_blobs=8)
    ms = (time.perf_counter() - t) * 1e3
    shares = [r / n for r in cr.ranges(1)]
    print(f"call {call:2d}: {ms:7.3f} ms  shares " + "  ".join(
        f"{name[:24]} {s:.3f}" for name, s in zip(cr.device_names(), shares)))
cr.dispose()
