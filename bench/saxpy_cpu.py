"""BASELINE config 1: float[1M] SAXPY on a single CPU device via compute()
(plumbing; runs without a GPU).  Checks bit-exactness against numpy."""
import argparse

import numpy as np

from common import emit, timeit

import cekirdekler_amd as ck

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1 << 20)
ap.add_argument("--reps", type=int, default=50)
a = ap.parse_args()
src = """__global__ void saxpy(const float* a, const float* x, float* y) {
    long long i = get_global_id(0); y[i] = a[0] * x[i] + y[i]; }"""
cr = ck.ClNumberCruncher(ck.AcceleratorType.CPU, src)
s = ck.ClArray(np.array([2.5], np.float32))
s.write = False
x = ck.ClArray(np.random.rand(a.n).astype(np.float32))
x.write = False
y0 = np.random.rand(a.n).astype(np.float32)
y = ck.ClArray(y0.copy())
s.next_param(x, y).compute(cr, 1, "saxpy", a.n, 256)
exact = bool(np.array_equal(y.array, np.float32(2.5) * x.array + y0))
ms = timeit(lambda: s.next_param(x, y).compute(cr, 1, "saxpy", a.n, 256), a.reps)
emit({"config": "saxpy_1M_cpu", "n": a.n, "ms": ms, "GBps": 12 * a.n / ms / 1e6,
      "bit_exact_vs_numpy": exact, "device": cr.device_names()[0]})
