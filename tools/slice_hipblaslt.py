"""GPU probe: torch (hipBLASLt) on the strongly scaled SGEMM slices
(rows x 8192 x 8192, bf16 in), median TF/s of 20-call runs, for context
next to tools/scale_probe.py: `a @ bt.T` (bf16 out, half our C bytes) and
`torch.mm(..., out_dtype=torch.float32)` (fp32 out, like ours).

    python tools/slice_hipblaslt.py [rows,...]
"""
import json
import statistics
import sys
import time

import torch

rows = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "8192,4096,2048,1024").split(",")]
out = {}
for m in rows:
    a = torch.randn(m, 8192, device="cuda", dtype=torch.bfloat16)
    bt = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    b = bt.T
    for name, fn in (("bf16_out", lambda: a @ b),
                     ("fp32_out", lambda: torch.mm(a, b, out_dtype=torch.float32))):
        try:
            for _ in range(5):
                c = fn()
        except Exception as e:  # out_dtype unsupported on this build
            out[f"{m}x8192x8192/{name}"] = {"error": str(e)[:120]}
            continue
        ts = []
        for _ in range(7):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                c = fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) / 20)
        med = statistics.median(ts)
        out[f"{m}x8192x8192/{name}"] = {"median_tflops": round(2 * m * 8192 * 8192 / med / 1e12, 1),
                                       "max_tflops": round(2 * m * 8192 * 8192 / min(ts) / 1e12, 1),
                                       "out_dtype": str(c.dtype)}
        del c
    del a, bt, b
print(json.dumps(out), flush=True)
