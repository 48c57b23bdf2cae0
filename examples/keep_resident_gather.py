"""Keep-resident iteration over several devices (ClArray.gather_resident).

A Jacobi-style smoothing step reads every neighbour, so after each step all
devices need everybody's slice.  The reference downloads every slice and
uploads the whole array on the next call (Tester.cs:7759-7765); with the
gather flag the slices are copied device→device after the kernels and
nothing crosses PCIe after the first call.

    python examples/keep_resident_gather.py          # every GPU (logical ×2 on one GPU)
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cekirdekler_amd as ck  # noqa: E402

SRC = """
__global__ void smooth(const float* x, float* y) {
  long long i = get_global_id(0), n = get_global_size(0);
  y[i] = 0.25f * x[(i + n - 1) % n] + 0.5f * x[i] + 0.25f * x[(i + 1) % n];
}
"""

plats = ck.ClPlatforms.all()
gpus = plats.gpus()
devs = (gpus[0] + gpus[0]) if len(gpus) == 1 else gpus if len(gpus) else plats.cpus(True) + plats.cpus(True)
cr = ck.ClNumberCruncher(devs, SRC)
n = 1 << 20
x0 = np.random.default_rng(0).standard_normal(n).astype(np.float32)
a, b = ck.ClArray(x0.copy()), ck.ClArray(np.zeros(n, np.float32))
for arr in (a, b):
    arr.write = False
src, dst = a, b
for it in range(20):
    src.read = it == 0            # uploaded once
    dst.read = False
    src.gather_resident, dst.gather_resident = False, True  # dst is written this step
    src.next_param(dst).compute(cr, 1, "smooth", n, 256)
    rec = cr.last_record()
    if it in (0, 1, 19):
        print(f"step {it}: h2d {rec['h2d_bytes']} B, d2h {rec['d2h_bytes']} B, "
              f"device->device {rec['p2p_bytes']} B ({rec['p2p_path']}), split {cr.ranges(1)}")
    src, dst = dst, src
cr.download(src, 0)               # every replica holds the whole result
ref = x0.astype(np.float64)
for _ in range(20):
    ref = 0.25 * np.roll(ref, 1) + 0.5 * ref + 0.25 * np.roll(ref, -1)
print("max |err| vs float64:", float(np.abs(src.array - ref).max()))
cr.dispose()
