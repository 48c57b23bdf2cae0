"""One process per GPU (torchrun): the global range is split across ranks by
the same load balancer; per-call timings are exchanged through shared memory,
so every rank derives the identical next split.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/distributed_saxpy.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np

import cekirdekler_amd as ck
from cekirdekler_amd.parallel.distributed import DistributedCruncher, init_distributed

SRC = "__global__ void saxpy(float* a, float* x, float* y) { long long i = get_global_id(0); y[i] = a[0] * x[i] + y[i]; }"
ctx = init_distributed()
cr = DistributedCruncher(SRC, ctx=ctx)
n = 1 << 24
a = ck.ClArray(np.array([2.0], np.float32)); a.write = False
x = ck.ClArray(np.ones(n, np.float32)); x.write = False
y = ck.ClArray(np.zeros(n, np.float32))
for _ in range(10):
    a.next_param(x, y).compute(cr, 1, "saxpy", n, 256)
lo = cr.references(1)[ctx.rank]
hi = lo + cr.ranges(1)[ctx.rank]
print(f"rank {ctx.rank}: items [{lo}, {hi}) ok={np.allclose(y.array[lo:hi], 20.0)} split={cr.ranges(1)}")
