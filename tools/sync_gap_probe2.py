import json, os, sys, time, statistics
sys.path.insert(0, os.getcwd())
import torch
import cekirdekler_amd as ck
from cekirdekler_amd.ops.gemm import GEMM_LIBS, GemmBf16
from cekirdekler_amd.ops.library import library
gpu = ck.ClPlatforms.all().gpus()[0]
cr = ck.ClNumberCruncher(gpu, "", prebuilt=library(*GEMM_LIBS), queue_concurrency=4)
g = GemmBf16(8192, 8192, 8192, cruncher=cr, tile="256x256pb")
for _ in range(10): g.run(compute_id=1, resident=True)
grp = g.dims.next_param(g.A, g.B, g.C, *g.extra)
call = cr._build_call(grp, 1, g.kernel, g.global_range, g.L, granularity=g.granularity())
core = cr._cores
out = {}
for name in ("native", "run"):
    w, rec = [], []
    for _ in range(30):
        t = time.perf_counter()
        if name == "native": core.compute(call)
        else: g.run(compute_id=1, resident=True)
        w.append((time.perf_counter() - t) * 1e3)
        rec.append(cr.last_record()["wall_ms"])
    out[name] = {"py_ms": round(statistics.median(w), 4), "native_wall_ms": round(statistics.median(rec), 4)}
# tiny kernel: native compute overhead without the GEMM
src = "__global__ void k(float* y) { long long i = get_global_id(0); y[i] = y[i] + 1.0f; }"
c2 = ck.ClNumberCruncher(gpu, src)
import numpy as np
y = ck.ClArray(1 << 14, np.float32); y.read = False; y.write = False
for _ in range(20): y.compute(c2, 7, "k", 1 << 14, 256)
w, rec = [], []
for _ in range(200):
    t = time.perf_counter(); y.compute(c2, 7, "k", 1 << 14, 256); w.append((time.perf_counter() - t) * 1e3); rec.append(c2.last_record()["wall_ms"])
out["tiny"] = {"py_ms": round(statistics.median(w), 4), "native_wall_ms": round(statistics.median(rec), 4)}
print(json.dumps(out), flush=True)
