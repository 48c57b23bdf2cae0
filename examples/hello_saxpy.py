"""Quick start: one kernel string, every device of a type, load-balanced.

    python examples/hello_saxpy.py            # GPUs if present, else the CPU device
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np

import cekirdekler_amd as ck

SRC = """
__kernel void saxpy(__global float* a, __global float* x, __global float* y)
{                                      // OpenCL-C dialect, as in the reference
    int i = get_global_id(0);
    y[i] = a[0] * x[i] + y[i];
}"""

plats = ck.ClPlatforms.all()
devices = plats.gpus() if len(plats.gpus()) else plats.cpus(True)
devices.log_info()
cr = ck.ClNumberCruncher(devices, SRC)
n = 1 << 22
a = ck.ClArray(np.array([2.0], np.float32)); a.write = False
x = ck.ClArray(np.random.rand(n).astype(np.float32)); x.write = False
y = ck.ClArray(n, np.float32)                      # pinned native array
y.array[:] = 1.0
for it in range(10):                               # same compute id → balancer converges
    a.next_param(x, y).compute(cr, 1, "saxpy", n, 256)
cr.performance_report(1)
print("ok:", np.allclose(y.array, 1.0 + 10 * 2.0 * x.array, rtol=1e-4))
cr.dispose()
