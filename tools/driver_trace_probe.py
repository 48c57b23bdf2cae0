"""GPU probe for a trace: the balanced LCG workload of bench/pipeline_overlap.py
(64 Mi uint32 in and out, ITERS steps per element) through the driver
pipeline (blob k on stream k mod Q) and the event pipeline, 16 blobs, two
calls each, outputs checked.  Run under
``rocprofv3 --kernel-trace --memory-copy-trace`` and read the timeline with
tools/overlap_timeline.py.

    python tools/driver_trace_probe.py [iters] [Q]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pipeline_overlap import SRC, expected  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 1350
Q = int(sys.argv[2]) if len(sys.argv) > 2 else 0
n = 64 << 20
gpu = ck.ClPlatforms.all().gpus()[0]
cr = ck.ClNumberCruncher(gpu, SRC, **({"queue_concurrency": Q} if Q else {}))
x = ck.ClArray(n, np.uint32)
x.array[:] = np.random.default_rng(0).integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
x.partial_read = True
x.write = False
it = ck.ClArray(np.array([iters], np.int32))
it.write = False
y = ck.ClArray(n, np.uint32)
y.read = False
want = expected(x.array, iters)
for name, ptype, cid in (("driver", ck.PIPELINE_DRIVER, 1), ("event", ck.PIPELINE_EVENT, 2)):
    for k in range(3):
        y.array[:] = 0
        t = time.perf_counter()
        x.next_param(it, y).compute(cr, cid, "lcg", n, 256, 0, True, ptype, 16)
        ms = (time.perf_counter() - t) * 1e3
        print(name, k, round(ms, 3), bool(np.array_equal(y.array, want)), flush=True)
cr.dispose()
