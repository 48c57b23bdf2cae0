"""GPU probe: host-resident SGEMM 8192³ (A, B uploaded and C downloaded on
every call) — serial 3-phase vs the event-driven streamed pipeline with
several blob counts.  Checks the streamed C against a float64 host product
on sampled tiles."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.ops.gemm import GEMM_LIBS, GemmBf16, tile_coords  # noqa: E402
from cekirdekler_amd.ops.library import library  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
blob_list = [int(b) for b in (sys.argv[2] if len(sys.argv) > 2 else "0,2,4,8").split(",")]
opts = sys.argv[3].split(",") if len(sys.argv) > 3 else []
resident_first = "resident-first" in opts
if "torch-first" in opts:  # initialise torch's HIP state first, as bench.py does
    import torch
    torch.cuda.synchronize()
reps = 5
if "dist" in opts:
    from cekirdekler_amd.parallel.distributed import DistributedCruncher
    cr = DistributedCruncher("", prebuilt=library(*GEMM_LIBS))
else:
    cr = ck.ClNumberCruncher(ck.ClPlatforms.all().gpus()[0], "", prebuilt=library(*GEMM_LIBS))
g = GemmBf16(size, size, size, cruncher=cr, tile="256x256pb")
sync_each = "sync-each" in opts
cr.cores.pipeline_writes_on_compute_stream = "wcs" in opts
if "npC" in opts:  # C in plain (registered) host memory instead of hipHostMalloc
    e = g.C.elements_per_work_item
    g.C = ck.ClArray(np.zeros(size * size, np.float32))
    g.C.read = False
    g.C.elements_per_work_item = e
if "npAB" in opts:
    for nm in ("A", "B"):
        old = getattr(g, nm)
        new = ck.ClArray(old.array.copy())
        new.write = False
        setattr(g, nm, new)
hip_sync_each = "hipsync-each" in opts
finish_each = "finish-each" in opts
if resident_first:  # the bench's order: device-resident computes in enqueue mode first
    for _ in range(10):
        g.run(compute_id=1, resident=True)
    cr.enqueue_mode = True
    for _ in range(20):
        g.run(compute_id=1, resident=True)
    cr.enqueue_mode = False
if "verify-first" in opts:
    g.run(compute_id=1, resident=True)
    print("verify", g.verify(compute_id=1), flush=True)
out = {}
for cid, blobs in enumerate(blob_list, start=10):
    g.C.array[:] = 0
    g.run(compute_id=cid, resident=False, stream_blobs=blobs, stream_event="driver" not in opts)  # warm
    ts = []
    for _ in range(reps):
        if sync_each:
            import torch
            torch.cuda.synchronize()
        if hip_sync_each:
            from cekirdekler_amd import cek
            cek.device_synchronize(0)
        if finish_each:
            cr.cores.finish()
        t = time.perf_counter()
        g.run(compute_id=cid, resident=False, stream_blobs=blobs, stream_event="driver" not in opts)
        if "finish-in" in opts:
            cr.cores.finish()  # inside the timed region: anything still in flight is counted
        ts.append((time.perf_counter() - t) * 1e3)
    # sampled check of the host C written by the last call
    rng = np.random.default_rng(cid)
    a = (g.A.array.astype(np.uint32) << 16).view(np.float32).reshape(size, size)
    b = (g.B.array.astype(np.uint32) << 16).view(np.float32).reshape(size, size)
    picks = rng.choice(g.tiles, 6, replace=False)
    tm, tn = tile_coords(picks, size, size, g.BM, g.BN, g.group_m)
    err = 0.0
    for t, r, c in zip(picks, tm, tn):
        got = g.tile_block(g.C.array[t * g.BM * g.BN:(t + 1) * g.BM * g.BN])
        ref = a[r * g.BM:(r + 1) * g.BM].astype(np.float64) @ b[c * g.BN:(c + 1) * g.BN].astype(np.float64).T
        err = max(err, float(np.abs(got - ref).max() / np.abs(ref).max()))
    rec = cr.last_record()
    out[f"blobs={blobs}"] = {"ms_median": float(np.median(ts)), "ms_min": float(min(ts)), "ms_all": ts,
                             "tflops": 2 * size ** 3 / (np.median(ts) * 1e-3) / 1e12, "max_rel_err": err,
                             "pipelined": rec["pipelined"], "h2d_MiB": rec["h2d_bytes"] / 2 ** 20,
                             "d2h_MiB": rec["d2h_bytes"] / 2 ** 20}
    print(json.dumps({f"blobs={blobs}": out[f"blobs={blobs}"]}), flush=True)
cr.dispose()
