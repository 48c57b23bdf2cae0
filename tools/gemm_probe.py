"""GPU probe: time the AOT GEMM kernels through compute() vs torch.matmul."""
import sys, time, json
sys.path.insert(0, '.')
import numpy as np
import torch
import cekirdekler_amd as ck
from cekirdekler_amd.ops.gemm import GemmBf16

res = {}
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
g0 = ck.ClPlatforms.all().gpus()[0]
import os
rows = [int(x) for x in os.environ.get("GEMM_PROBE_ROWS", "").split(",") if x]
shapes = [(r, n, n) for r in rows] if rows else [(n, n, n)] + ([(n // 8, n, n)] if n >= 4096 else [])
from cekirdekler_amd.ops.gemm import TILES
tiles = sys.argv[2].split(",") if len(sys.argv) > 2 else list(TILES)
groups = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 4, 8]
for (M, N, K), tile, gm in [(s, t, g) for s in shapes for t in tiles for g in groups]:
    tname, _, sk = tile.partition(":s")
    g = GemmBf16(M, N, K, devices=g0, tile=tname, group_m=gm, split_k=int(sk or 1))
    for _ in range(3): g.run(resident=True)
    torch.cuda.synchronize()
    t = time.perf_counter(); REPS = 20
    for _ in range(REPS): g.run(resident=True)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1e3 / REPS
    key = f"{M}x{N}x{K}/{tile}/g{gm}"
    res[key] = {"ms": ms, "tflops": g.flops / ms / 1e9, "dev_ms": g.cr.benchmarks(1)}
    if n <= 8192:
        rows = slice(0, 256)
        c = g.result(download=True)[rows]
        ref = g.reference(rows)
        res[key]["max_err"] = float(np.abs(c - ref).max())
    g.cr.dispose()
a = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
b = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
for _ in range(3): torch.matmul(a, b.t())
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(20): torch.matmul(a, b.t())
torch.cuda.synchronize(); ms = (time.perf_counter() - t) * 1e3 / 20
res["torch_bf16_nt"] = {"ms": ms, "tflops": 2 * n**3 / ms / 1e9}
print(json.dumps(res, indent=1))
