"""GPU probe: does one device-wide sync leave the streamed host-resident
SGEMM (event pipeline, 8 blobs) slow for every later call?  Times each call
through phases: back to back; after an idle pause; after one
hipDeviceSynchronize; on a fresh cruncher (new streams); after a sync on
that one.  See profiles/hostres_streaming.md.

    python tools/hostres_stall_probe.py [blobs] [calls_per_phase] [kd2h]

``kd2h``: downloads by the runtime's copy kernel (``kernel_d2h``) instead of
hipMemcpyAsync.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd import cek  # noqa: E402
from cekirdekler_amd.ops.gemm import GEMM_LIBS, GemmBf16, from_bf16_bits, tile_coords  # noqa: E402
import numpy as np  # noqa: E402
from cekirdekler_amd.ops.library import library  # noqa: E402

blobs = int(sys.argv[1]) if len(sys.argv) > 1 else 8
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 6
kd2h = "kd2h" in sys.argv[3:]
size = 8192
dev = ck.ClPlatforms.all().gpus()[0]


def make():
    cr = ck.ClNumberCruncher(dev, "", prebuilt=library(*GEMM_LIBS))
    cr.kernel_d2h = kd2h
    cr.cores.pipeline_reads_on_main_stream = "rms" in sys.argv[3:]
    cr.cores.pipeline_writes_on_compute_stream = "wcs" in sys.argv[3:]
    return GemmBf16(size, size, size, cruncher=cr, tile="256x256pb")


def phase(g, name, out):
    ts = []
    for _ in range(calls):
        t = time.perf_counter()
        g.run(compute_id=2, resident=False, stream_blobs=blobs)
        ts.append(round((time.perf_counter() - t) * 1e3, 3))
    out[name] = ts
    print(name, ts, flush=True)


out = {}
g = make()
g.run(compute_id=2, resident=False, stream_blobs=blobs)  # warm
phase(g, "back_to_back", out)
time.sleep(0.2)
phase(g, "after_idle_200ms", out)
cek.device_synchronize(0)
phase(g, "after_one_device_sync", out)
g.cr.cores.finish()
phase(g, "after_cores_finish", out)
g2 = make()
g2.run(compute_id=2, resident=False, stream_blobs=blobs)  # warm
phase(g2, "fresh_cruncher", out)
cek.device_synchronize(0)
phase(g2, "fresh_after_device_sync", out)
# the last call's host C against a float64 product on sampled tiles
rng = np.random.default_rng(0)
a = from_bf16_bits(g2.A.array).reshape(size, size)
b = from_bf16_bits(g2.B.array).reshape(size, size)
picks = rng.choice(g2.tiles, 4, replace=False)
tm, tn = tile_coords(picks, size, size, g2.BM, g2.BN, g2.group_m)
err = 0.0
for t, r, c in zip(picks, tm, tn):
    got = g2.tile_block(g2.C.array[t * g2.BM * g2.BN:(t + 1) * g2.BM * g2.BN])
    ref = a[r * g2.BM:(r + 1) * g2.BM].astype(np.float64) @ b[c * g2.BN:(c + 1) * g2.BN].astype(np.float64).T
    err = max(err, float(np.abs(got - ref).max() / np.abs(ref).max()))
out["max_rel_err"] = err
out["kernel_d2h"] = kd2h
out["opts"] = sys.argv[3:]
out["kernel_d2h_MiB"] = g2.cr.cores.kernel_d2h_bytes / 2 ** 20
print(json.dumps(out), flush=True)
g.cr.dispose()
g2.cr.dispose()
