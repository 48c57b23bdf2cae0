"""GPU probe: Mandelbrot 4096² end to end with the image as a zero-copy
array (the kernel's stores go straight over PCIe into pinned host memory,
no D2H copies) against the event pipeline (8 blobs, SDMA D2H).  Median of
15 calls; every variant's image is compared with the pipeline's."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.models.mandelbrot import MandelbrotRenderer  # noqa: E402

kernels = sys.argv[1].split(",") if len(sys.argv) > 1 else ["blk8"]
gpu = ck.ClPlatforms.all().gpus()[0]
res = {}


def med(fn, n=15):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t) * 1e3)
    return round(sorted(ts)[n // 2], 4)


for kern in kernels:
    m = MandelbrotRenderer(4096, 4096, 256, devices=gpu, kernel=kern)
    res[f"{kern}/pipeline_b8"] = med(lambda: m.render(1, pipeline=True, blobs=8))
    ref = m.out.array.copy()
    e = m.out.elements_per_work_item
    for kind in ("hostmalloc", "registered"):
        out = ck.ClArray(4096 * 4096, np.int32) if kind == "hostmalloc" else ck.ClArray(np.zeros(4096 * 4096, np.int32))
        out.read = False
        out.elements_per_work_item = e
        out.zero_copy = True
        m.out = out
        res[f"{kern}/zero_copy_{kind}"] = med(lambda: m.render(2 if kind == "hostmalloc" else 3, pipeline=False))
        res[f"{kern}/zero_copy_{kind}_equal"] = bool(np.array_equal(out.array, ref))
    m.cr.dispose()
print(json.dumps(res), flush=True)
