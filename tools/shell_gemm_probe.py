"""GPU probe: host-resident SGEMM 8192³ (A, B up and C down every call)
streamed in square shells (``GemmBf16.run_host_shells``) for several panel
counts, against the 1-D blob pipeline (``run(resident=False,
stream_blobs=8)``).  Each variant: 2 warm calls, a device sync, then
``calls`` timed calls; sampled check against float64.

    python tools/shell_gemm_probe.py [panels,...] [calls] [tile] [kd2h]
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd import cek  # noqa: E402
from cekirdekler_amd.ops.gemm import GEMM_LIBS, GemmBf16  # noqa: E402
from cekirdekler_amd.ops.library import library  # noqa: E402

panel_list = [int(p) for p in (sys.argv[1] if len(sys.argv) > 1 else "4,8,16").split(",")]
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 8
tile = sys.argv[3] if len(sys.argv) > 3 else "256x256pb"
size = 8192
cr = ck.ClNumberCruncher(ck.ClPlatforms.all().gpus()[0], "", prebuilt=library(*GEMM_LIBS))
g = GemmBf16(size, size, size, cruncher=cr, tile=tile)
# wcs: downloads on the compute streams, right behind each shell's kernels
cr.cores.pipeline_writes_on_compute_stream = "wcs" in sys.argv[4:]
out = {}


def timed(fn):
    for _ in range(2):
        fn()
    cek.device_synchronize(0)
    ts = []
    for _ in range(calls):
        t = time.perf_counter()
        fn()
        ts.append(round((time.perf_counter() - t) * 1e3, 3))
    return ts


ts = timed(lambda: g.run(compute_id=2, resident=False, stream_blobs=8))
out["blobs8"] = {"ms_median": statistics.median(ts), "ms": ts, "max_rel_err": g.verify(compute_id=2, host=True)}
print(json.dumps({"blobs8": out["blobs8"]}), flush=True)
for p in panel_list:
    ts = timed(lambda: g.run_host_shells(p))
    out[f"shells{p}"] = {"ms_median": statistics.median(ts), "ms": ts, "max_rel_err": g.verify_shells(p)}
    print(json.dumps({f"shells{p}": out[f"shells{p}"]}), flush=True)
if "kd2h" in sys.argv[4:]:
    # the same shells with downloads by the runtime's copy kernel (D2H off the SDMA / blit path)
    cr.kernel_d2h = True
    for p in panel_list:
        ts = timed(lambda: g.run_host_shells(p))
        out[f"shells{p}_kd2h"] = {"ms_median": statistics.median(ts), "ms": ts, "max_rel_err": g.verify_shells(p)}
        print(json.dumps({f"shells{p}_kd2h": out[f"shells{p}_kd2h"]}), flush=True)
for k, v in out.items():
    v["tflops"] = round(2 * size ** 3 / (v["ms_median"] * 1e-3) / 1e12, 1)
print(json.dumps(out), flush=True)
cr.dispose()
