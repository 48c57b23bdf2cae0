"""GPU probe: Mandelbrot 4096² kernel-only frames rendered back to back in
enqueue mode, one stream (the bench's kernel-only method) against the
reference's async enqueue mode (enqueueModeAsyncEnable: each compute() on
the next of the cruncher's queues), where frame k+1's first waves can start
while frame k's last waves finish.  Two renderers (two output images,
compute ids 1 and 2) alternate, so overlapping frames never write the same
buffer.

    python tools/mandel_async_probe.py [rounds] [frames]
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
from cekirdekler_amd.ops.library import library  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 20
gpu = ck.ClPlatforms.all().gpus()[0]
cr = ck.ClNumberCruncher(gpu, "", prebuilt=library("mandelbrot"), queue_concurrency=2)
ms = [MandelbrotRenderer(4096, 4096, 256, cruncher=cr, kernel="blk8y") for _ in range(2)]
for i, m in enumerate(ms):
    m.render(i + 1, pipeline=False)
flops = ms[0].flops()
for m in ms:
    m.out.write = False
ref = ms[0].out.array.copy()
res = {"sync_stream": [], "async_queues": []}
for _ in range(rounds):
    for mode in res:
        cr.enqueue_mode_async_enable = mode == "async_queues"
        for k in range(40):
            ms[k & 1].render((k & 1) + 1, pipeline=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cr.enqueue_mode = True
        for k in range(frames):
            ms[k & 1].render((k & 1) + 1, pipeline=False)
        cr.enqueue_mode = False
        torch.cuda.synchronize()
        res[mode].append((time.perf_counter() - t0) * 1e3 / frames)
cr.enqueue_mode_async_enable = False
ok = True
for m in ms:  # the device images the overlapped frames wrote last
    m.out.array[:] = -1
    cr.download(m.out, 0)
    ok = ok and bool((m.out.array == ref).all())
out = {"frames": frames, "rounds": rounds, "images_equal": ok, "queues": cr.compute_queue_concurrency}
for mode, v in res.items():
    med = statistics.median(v)
    out[mode] = {"ms_median": round(med, 4), "ms_min": round(min(v), 4),
                 "pct_fp32_peak": round(100 * flops / (med * 1e-3) / 1e12 / 157.3, 1)}
print(json.dumps(out))
cr.dispose()
