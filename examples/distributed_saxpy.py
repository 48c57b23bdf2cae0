"""One process per GPU (torchrun): the global range is split across ranks by
the same load balancer; per-call timings are exchanged through shared memory,
so every rank derives the identical next split.

Each rank has its own host copy of every array and receives only its own
slices of the written ones.  An array that is read whole AND written by
slices (``y = a*x + y`` over many calls) is therefore coherent only with the
RCCL data plane: ``DistributedCruncher(comm=True)`` + ``gather_writes``
all-gathers the written slices over xGMI into every replica (and host copy).
Without one GPU per rank (e.g. two ranks sharing a GPU) this example
computes ``y = a*x + 1`` instead, which needs no coherence.

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
rccl = ctx.backend == "nccl"  # one GPU per rank
cr = DistributedCruncher(SRC, ctx=ctx, comm=rccl)
if rccl:
    cr.gather_writes = True
n = 1 << 24
a = ck.ClArray(np.array([2.0], np.float32)); a.write = False
x = ck.ClArray(np.ones(n, np.float32)); x.write = False
y = ck.ClArray(np.zeros(n, np.float32))
if not rccl:
    y.partial_read = True  # each rank uploads exactly the slice it computes
for _ in range(10):
    if not rccl:
        y.array[:] = 1.0  # y = a*x + 1: a fresh addend every call
    a.next_param(x, y).compute(cr, 1, "saxpy", n, 256)
want = 20.0 if rccl else 3.0
lo = cr.references(1)[ctx.rank]
hi = lo + cr.ranges(1)[ctx.rank]
full = bool(np.allclose(y.array, want)) if rccl else None
print(f"rank {ctx.rank}: items [{lo}, {hi}) ok={np.allclose(y.array[lo:hi], want)} whole array ok={full} "
      f"split={cr.ranges(1)}")
