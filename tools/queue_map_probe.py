"""GPU probe: which async compute streams of a fresh cruncher share a
hardware queue.  Eight long one-wave-per-CU kernels are enqueued back to back
in async enqueue mode (compute k on stream k mod Q); the hipEvent timeline
shows which consecutive computes ran side by side (distinct hardware queues)
and which ran one after the other (one queue)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cekirdekler_amd as ck  # noqa: E402

Q = int(sys.argv[1]) if len(sys.argv) > 1 else 4
src = ("__global__ void spin(float* y) { long long i = get_global_id(0); float v = y[i];"
       " for (int j = 0; j < 200000; ++j) v = v * 0.9999f + 0.5f; y[i] = v; }")
gpu = ck.ClPlatforms.all().gpus()
cr = ck.ClNumberCruncher(gpu[0], src, queue_concurrency=Q)
ys = [ck.ClArray(1 << 14, np.float32) for _ in range(8)]
for y in ys:
    y.read = y.write = False
    y.compute(cr, 1, "spin", 1 << 14, 256)  # buffers, warm
runs = []
for rep in range(2):
    cr.record_timeline = True
    cr.enqueue_mode = True
    cr.enqueue_mode_async_enable = True
    for k, y in enumerate(ys):
        y.compute(cr, 10 + k, "spin", 1 << 14, 256)
    cr.enqueue_mode = False
    cr.enqueue_mode_async_enable = False
    tl = sorted(cr.timeline(), key=lambda t: t["compute_id"])
    runs.append([(t["compute_id"] - 10, round(t["begin_ms"], 3), round(t["end_ms"], 3)) for t in tl])
    cr.record_timeline = False
print(json.dumps({"Q": Q, "runs": runs}), flush=True)
cr.dispose()
