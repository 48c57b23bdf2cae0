"""Calls of the balanced read/compute/write workload (bench/pipeline_overlap.py)
for a timeline under rocprofv3: the 3-phase path once, then the driver
pipeline (16 blobs, default compute streams) four times; the last driver
call is the one summarised by tools/trace_overlap.py.

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d OUT -o run \
        -- python3 tools/driver_pipeline_trace.py [--iters 1338]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench"))
import cekirdekler_amd as ck  # noqa: E402
from pipeline_overlap import SRC, expected  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=64 << 20)
ap.add_argument("--iters", type=int, default=1338)
ap.add_argument("--blobs", type=int, default=16)
a = ap.parse_args()

dev = ck.ClPlatforms.all().gpus()[0]
n = a.n
rng = np.random.default_rng(0)
x = ck.ClArray(n, np.uint32)
x.array[:] = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
x.partial_read = True
x.write = False
it = ck.ClArray(np.array([a.iters], np.int32))
it.write = False
y = ck.ClArray(n, np.uint32)
y.read = False
cr = ck.ClNumberCruncher(dev, SRC)
x.next_param(it, y).compute(cr, 1, "lcg", n, 256)  # 3-phase
for _ in range(4):
    x.next_param(it, y).compute(cr, 2, "lcg", n, 256, 0, True, ck.PIPELINE_DRIVER, a.blobs)
ok = bool(np.array_equal(y.array, expected(x.array, a.iters)))
print({"exact": ok, "blobs": a.blobs, "iters": a.iters, "streams": cr.compute_queue_concurrency}, flush=True)
cr.dispose()
