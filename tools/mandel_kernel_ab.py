"""GPU probe: Mandelbrot 4096² kernel-only time (image left in device
memory), variants interleaved over rounds in one process, median and min
per variant; FLOPs from the escape counts (8 per iteration).  The timed
calls run in enqueue mode (back to back, no host sync per call), as in
bench.py's kernel-only number; ``sync_ms_median`` is the same with a host
sync per call.

    python tools/mandel_kernel_ab.py blk8h,blk8k,blk8t [rounds] [reps]
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.models.mandelbrot import MandelbrotRenderer  # noqa: E402

kernels = sys.argv[1].split(",")
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 7
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
gpu = ck.ClPlatforms.all().gpus()[0]
rs, flops = {}, {}
for k in kernels:
    m = MandelbrotRenderer(4096, 4096, 256, devices=gpu, kernel=k)
    m.render(1, pipeline=False)
    flops[k] = m.flops()
    m.out.write = False
    rs[k] = m
ts = {k: [] for k in kernels}
sync_ts = {k: [] for k in kernels}
for r in range(rounds):
    for k, m in rs.items():
        for _ in range(3):
            m.render(1, pipeline=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            m.render(1, pipeline=False)
        torch.cuda.synchronize()
        sync_ts[k].append((time.perf_counter() - t0) * 1e3 / reps)
        t0 = time.perf_counter()
        m.cr.enqueue_mode = True
        for _ in range(reps):
            m.render(1, pipeline=False)
        m.cr.enqueue_mode = False
        torch.cuda.synchronize()
        ts[k].append((time.perf_counter() - t0) * 1e3 / reps)
out = {}
for k in kernels:
    med = statistics.median(ts[k])
    out[k] = {"ms_median": round(med, 4), "ms_min": round(min(ts[k]), 4),
              "tflops_median": round(flops[k] / med / 1e9, 2),
              "pct_fp32_peak_median": round(flops[k] / med / 1e9 / 157.3 * 100, 1),
              "sync_ms_median": round(statistics.median(sync_ts[k]), 4)}
print(json.dumps(out), flush=True)
