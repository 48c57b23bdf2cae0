"""GPU probe: Mandelbrot 4096² end to end through the event pipeline, by
where the blob downloads are issued — the two halves' write streams
(default), one write stream for every blob (``pipeline_writes_one_stream``)
or each blob's compute stream — and by blob count.  Each variant: a device
sync, then 15 timed renders (median).

    python tools/mandel_ws_probe.py [blobs,...]
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd import cek  # noqa: E402
from cekirdekler_amd.models.mandelbrot import MandelbrotRenderer  # noqa: E402

blob_list = [int(b) for b in (sys.argv[1] if len(sys.argv) > 1 else "4,8,16").split(",")]
m = MandelbrotRenderer(4096, 4096, 256, devices=ck.ClPlatforms.all().gpus()[0])
ref = None
out = {}
cid = 100
for mode in ("two", "one", "wcs"):
    m.cr.cores.pipeline_writes_one_stream = mode == "one"
    m.cr.cores.pipeline_writes_on_compute_stream = mode == "wcs"
    for blobs in blob_list:
        cid += 1
        for _ in range(3):
            img = m.render(cid, pipeline=True, blobs=blobs)
        if ref is None:
            ref = img.copy()
        ok = bool((img == ref).all())
        cek.device_synchronize(0)
        ts = []
        for _ in range(15):
            t = time.perf_counter()
            m.render(cid, pipeline=True, blobs=blobs)
            ts.append((time.perf_counter() - t) * 1e3)
        out[f"{mode}_b{blobs}"] = {"ms_median": round(statistics.median(ts), 4), "ms_min": round(min(ts), 4),
                                   "same_image": ok}
        print(json.dumps({f"{mode}_b{blobs}": out[f"{mode}_b{blobs}"]}), flush=True)
print(json.dumps(out), flush=True)
