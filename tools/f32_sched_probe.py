"""GPU probe: the fp32 GEMM code object built with different LLVM machine
schedulers (``-mllvm -amdgpu-sched-strategy=...``), same source, timed
through compute() in interleaved rounds.

    python tools/f32_sched_probe.py variant.hsaco,... [tile] [rounds]
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402
import cekirdekler_amd.ops.gemm as gemm  # noqa: E402
import cekirdekler_amd.ops.library as lib  # noqa: E402

paths = sys.argv[1].split(",")
tile = sys.argv[2] if len(sys.argv) > 2 else "256x256ir"
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dev = ck.ClPlatforms.all().gpus()[0]
orig = lib.code_object
runs = {}
for p in paths:
    lib.code_object = lambda name, p=p: os.path.abspath(p) if name == "sgemm_f32" else orig(name)
    gemm.library = lib.library
    runs[p] = gemm.GemmF32(8192, 8192, 8192, devices=dev, tile=tile)
    runs[p].run(resident=True)
lib.code_object = orig
res = {p: [] for p in paths}
for _ in range(rounds):
    for p, g in runs.items():
        for _ in range(2):
            g.run(resident=True)
        torch.cuda.synchronize()
        t = time.perf_counter()
        g.cr.enqueue_mode = True
        for _ in range(5):
            g.run(resident=True)
        g.cr.enqueue_mode = False
        torch.cuda.synchronize()
        res[p].append(g.flops / ((time.perf_counter() - t) / 5) / 1e12)
out = {os.path.basename(p): round(statistics.median(v), 1) for p, v in res.items()}
for p, g in runs.items():
    rows = slice(0, 128)
    c = g.result(download=True)[rows]
    ref = g.reference(rows)
    out[os.path.basename(p) + "_err"] = float(abs(c - ref).max() / abs(ref).max())
print(json.dumps(out))
