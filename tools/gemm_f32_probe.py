"""GPU probe: fp32 matrix-core GEMM tiles through compute() (enqueue mode,
interleaved rounds) vs torch.matmul fp32 (hipBLASLt) on the same shape.

    python tools/gemm_f32_probe.py [n] [tile,...] [rounds] [steps]
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.ops.gemm import GemmF32  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
tiles = (sys.argv[2] if len(sys.argv) > 2 else "128x128,256x128,256x256").split(",")
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
dev = ck.ClPlatforms.all().gpus()[0]
# a tile may carry its tile-group height: "256x256ir@8"
runs = {t: GemmF32(n, n, n, devices=dev, tile=t.split("@")[0], group_m=int(t.split("@")[1]) if "@" in t else 4)
        for t in tiles}
for g in runs.values():
    g.run(resident=True)
torch.backends.cuda.matmul.allow_tf32 = False
a = torch.from_numpy(runs[tiles[0]].A.array.reshape(n, n)).cuda()
b = torch.from_numpy(runs[tiles[0]].B.array.reshape(n, n)).cuda()
torch.matmul(a, b.t())
torch.cuda.synchronize()
res = {t: [] for t in tiles}
res["torch_fp32_nt"] = []
for _ in range(rounds):
    for t, g in runs.items():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.cr.enqueue_mode = True
        for _ in range(steps):
            g.run(resident=True)
        g.cr.enqueue_mode = False
        torch.cuda.synchronize()
        res[t].append(g.flops / ((time.perf_counter() - t0) * 1e3 / steps) / 1e9)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        torch.matmul(a, b.t())
    torch.cuda.synchronize()
    res["torch_fp32_nt"].append(2 * n ** 3 / ((time.perf_counter() - t0) * 1e3 / steps) / 1e9)
out = {k: {"median_tflops": round(statistics.median(v), 1), "max_tflops": round(max(v), 1)} for k, v in res.items()}
for t, g in runs.items():
    c = g.result(download=True)[:128]
    out[t]["max_rel_err_rows0_127"] = float(abs(c - g.reference(slice(0, 128))).max() / abs(c).max())
print(json.dumps(out, indent=1))
