"""GPU probe: Mandelbrot 4096² kernel variants end to end through the event
pipeline (8 blobs), interleaved over rounds on one box (median ms), plus
each variant's pixel mismatch against the float32 numpy reference on the
first 1024 rows.

    python tools/mandel_ab_probe.py blk8,blk8h,blk8t [rounds] [blobs,...]
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.models.mandelbrot import MandelbrotRenderer  # noqa: E402

kernels = sys.argv[1].split(",")
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
blob_list = [int(b) for b in (sys.argv[3] if len(sys.argv) > 3 else "8").split(",")]
gpu = ck.ClPlatforms.all().gpus()[0]
ms = {(k, b): [] for k in kernels for b in blob_list}
rs = {k: MandelbrotRenderer(4096, 4096, 256, devices=gpu, kernel=k) for k in kernels}
for r in range(rounds):
    for (k, b) in ms:
        m = rs[k]
        cid = 1 + b  # one compute id (own balancer state) per blob count
        for _ in range(2):
            m.render(cid, pipeline=True, blobs=b)
        ts = []
        for _ in range(10):
            t = time.perf_counter()
            m.render(cid, pipeline=True, blobs=b)
            ts.append((time.perf_counter() - t) * 1e3)
        ms[(k, b)].append(statistics.median(ts))
ref = next(iter(rs.values())).reference(rows=1024)
out = {}
for (k, b), v in ms.items():
    img = rs[k].out.array.reshape(4096, 4096)[:1024]
    out[f"{k}/b{b}"] = {"e2e_ms_median": round(statistics.median(v), 4), "e2e_ms_min": round(min(v), 4),
                        "mismatch_vs_numpy_rows0_1023": float(np.mean(img != ref))}
print(json.dumps(out), flush=True)
