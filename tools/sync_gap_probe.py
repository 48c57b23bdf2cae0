"""GPU probe: where a synchronous compute() of the headline GEMM (8192³ bf16,
device-resident) spends the time beyond its kernel.  Per call: host wall
time, the kernel's dispatch-stamped time, and a cProfile of the Python side;
the same K calls in enqueue mode for comparison.

    python tools/sync_gap_probe.py [calls]
"""
import cProfile
import io
import json
import os
import pstats
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.ops.gemm import GEMM_LIBS, GemmBf16  # noqa: E402
from cekirdekler_amd.ops.library import library  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
gpu = ck.ClPlatforms.all().gpus()[0]
cr = ck.ClNumberCruncher(gpu, "", prebuilt=library(*GEMM_LIBS), queue_concurrency=4)
g = GemmBf16(8192, 8192, 8192, cruncher=cr, tile="256x256pb")
for _ in range(10):
    g.run(compute_id=1, resident=True)
torch.cuda.synchronize()
walls = []
for _ in range(K):
    t = time.perf_counter()
    g.run(compute_id=1, resident=True)
    walls.append((time.perf_counter() - t) * 1e3)
cr.record_kernel_times = True
for _ in range(K):
    g.run(compute_id=1, resident=True)
cr.record_kernel_times = False
kt = [ms for name, ms in cr.kernel_times(0) if name.startswith("cek_sgemm")]
t = time.perf_counter()
cr.enqueue_mode = True
for _ in range(K):
    g.run(compute_id=1, resident=True)
cr.enqueue_mode = False
torch.cuda.synchronize()
enq = (time.perf_counter() - t) * 1e3 / K
pr = cProfile.Profile()
pr.enable()
for _ in range(K):
    g.run(compute_id=1, resident=True)
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(14)
rec = cr.last_record()
print(json.dumps({"sync_wall_ms_median": round(statistics.median(walls), 4),
                  "sync_wall_ms": [round(x, 4) for x in walls],
                  "kernel_ms_median": round(statistics.median(kt), 4) if kt else None,
                  "enqueue_ms_per_call": round(enq, 4),
                  "last_record": {k: rec.get(k) for k in ("wall_ms", "device_ms")},
                  "profile": s.getvalue()[-3500:]}), flush=True)
cr.dispose()
