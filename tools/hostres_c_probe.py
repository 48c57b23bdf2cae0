"""Host-resident SGEMM 8192³: where C's host pages
live decides which engine downloads it.

Into ``hipHostMalloc`` memory (a FastArr, the GemmBf16 default) the runtime
downloads with ``__amd_rocclr_copyBuffer`` blit kernels on the CUs, beside
the GEMM; into registered pages (numpy + ``hipHostRegister``) it uses an
SDMA engine (profiles/hostres_streaming.md, the Mandelbrot renderer's
choice).  This probe times the square-shell stream through compute()
(``run_shells``, 16 panels) and the 8-blob row-panel stream with C in each
kind of memory, rounds interleaved, and checks every C tile of each
(``verify_full``).

    python tools/hostres_c_probe.py [rounds] > gpurun_out/hostres_c.json
"""
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.arrays import ClArray  # noqa: E402
from cekirdekler_amd.ops.gemm import GEMM_LIBS, GemmBf16  # noqa: E402
from cekirdekler_amd.ops.library import library  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
gpu = ck.ClPlatforms.all().gpus()[0]
cr = ck.ClNumberCruncher(gpu, "", prebuilt=library(*GEMM_LIBS))
S = 8192
g = GemmBf16(S, S, S, cruncher=cr, tile="256x256pb")
c_fast = g.C
c_reg = ClArray(np.zeros(S * S, np.float32))
c_reg.read = False
c_reg.elements_per_work_item = c_fast.elements_per_work_item


def use(c):
    g.C = c


configs = {
    "shells16_fastarr": (c_fast, lambda: g.run_shells(16, compute_id=3)),
    "shells16_registered": (c_reg, lambda: g.run_shells(16, compute_id=4)),
    "shells16_split2_registered": (c_reg, lambda: g.run_shells(16, compute_id=5, split_last=2)),
    "blobs8_fastarr": (c_fast, lambda: g.run(compute_id=6, resident=False, stream_blobs=8)),
    "blobs8_registered": (c_reg, lambda: g.run(compute_id=7, resident=False, stream_blobs=8)),
}
ids = {"shells16_fastarr": 3, "shells16_registered": 4, "shells16_split2_registered": 5, "blobs8_fastarr": 6,
       "blobs8_registered": 7}
times = {k: [] for k in configs}
errs = {}
for name, (c, fn) in configs.items():  # untimed: buffers, balancer state
    use(c)
    fn()
    fn()
    torch.cuda.synchronize()
    errs[name] = g.verify_full(compute_id=ids[name], host=True)
for _ in range(rounds):
    for name, (c, fn) in configs.items():
        use(c)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        times[name].append((time.perf_counter() - t0) * 1e3 / 3)
out = {"rounds": rounds, "ms": {k: round(statistics.median(v), 3) for k, v in times.items()},
       "ms_runs": {k: [round(x, 3) for x in v] for k, v in times.items()},
       "max_rel_err_full": {k: v[0] for k, v in errs.items()}, "tiles_checked": {k: v[1] for k, v in errs.items()}}
print(json.dumps(out), flush=True)
cr.dispose()
