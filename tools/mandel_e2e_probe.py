"""GPU probe: Mandelbrot 4096² end to end through the event pipeline, blob
counts × where the blob D2H is issued (write stream gated by an event, or
the blob's compute stream), with and without a device sync between calls."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.models.mandelbrot import MandelbrotRenderer  # noqa: E402

import numpy as np  # noqa: E402

m = MandelbrotRenderer(4096, 4096, 256, devices=ck.ClPlatforms.all().gpus()[0])
res = {}
if "np" in sys.argv[1:]:  # image in registered numpy memory instead of hipHostMalloc
    e = m.out.elements_per_work_item
    m.out = ck.ClArray(np.zeros(4096 * 4096, np.int32))
    m.out.read = False
    m.out.elements_per_work_item = e
for wcs in ((False,) if "np" in sys.argv[1:] else (False, True)):
    m.cr.cores.pipeline_writes_on_compute_stream = wcs
    for blobs in next((tuple(int(x) for x in a[6:].split(",")) for a in sys.argv[1:] if a.startswith("blobs=")),
                      (4, 8, 16)):
        for fin in (False, True):
            cid = 100 + blobs + (50 if wcs else 0)
            for _ in range(3):
                m.render(cid, pipeline=True, blobs=blobs)
            ts = []
            for _ in range(15):
                if fin:
                    m.cr.cores.finish()
                t = time.perf_counter()
                m.render(cid, pipeline=True, blobs=blobs)
                ts.append((time.perf_counter() - t) * 1e3)
            res[f"{'wcs' if wcs else 'ws'}_b{blobs}{'_fin' if fin else ''}"] = round(sorted(ts)[len(ts) // 2], 4)
print(json.dumps(res), flush=True)
