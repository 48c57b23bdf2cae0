"""GPU probe: the per-GPU share of the strongly scaled SGEMM 8192³ bench.

At N GPUs a rank computes ``8192/N`` rows of C (a contiguous tile range).  This
times that slice as a standalone ``rows × 8192 × 8192`` GEMM through
``compute()`` in enqueue mode — exactly the bench's timed loop — for several
tile kernels, interleaving the variants over rounds (one process, one device)
and reporting median / min TF/s.

    python tools/scale_probe.py [rows,...] [tile[:sS][:wD],...] [rounds] [steps]

(``:sS`` split-K S, ``:wD`` the helper's K-tile deficit of an uneven-split
tile, ``:a`` the computes on async enqueue queues — consecutive GEMMs overlap,
as the bench's async schedule runs them; ``:qN`` N async queues per device)
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.ops.gemm import GemmBf16  # noqa: E402

rows = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "8192,4096,2048,1024").split(",")]
tiles = (sys.argv[2] if len(sys.argv) > 2 else "256x256pb,256x128pe").split(",")
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
n = k = 8192
gm = int(os.environ.get("GEMM_GROUP_M", "4"))

dev = ck.ClPlatforms.all().gpus()[0]
runs = {}
for m in rows:
    for t in tiles:
        name, *opts = t.split(":")
        sk = next((int(o[1:]) for o in opts if o.startswith("s")), 1)
        wd = next((int(o[1:]) for o in opts if o.startswith("w")), None)
        asy = "a" in opts
        qc = next((int(o[1:]) for o in opts if o.startswith("q")), 0)  # async queues per device
        try:
            cr = None
            if qc:
                from cekirdekler_amd.ops.gemm import GEMM_LIBS
                from cekirdekler_amd.ops.library import library
                cr = ck.ClNumberCruncher(dev, "", prebuilt=library(*GEMM_LIBS), queue_concurrency=qc)
            g = GemmBf16(m, n, k, devices=dev, tile=name, group_m=gm, split_k=sk, exchange_shift=wd, cruncher=cr)
        except ValueError as e:
            print(f"skip {m}/{t}: {e}", flush=True)
            continue
        for _ in range(3):
            g.run(resident=True)
        if asy:  # create the async queues' streams before timing
            g.cr.enqueue_mode = True
            g.cr.enqueue_mode_async_enable = True
            for _ in range(g.cr.compute_queue_concurrency + 1):
                g.run(resident=True)
            g.cr.enqueue_mode = False
            g.cr.enqueue_mode_async_enable = False
        g.async_queues = asy
        runs[(m, t)] = g
torch.cuda.synchronize()

res = {key: [] for key in runs}
for r in range(rounds):
    for key, g in runs.items():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.cr.enqueue_mode = True
        g.cr.enqueue_mode_async_enable = g.async_queues
        for _ in range(steps):
            g.run(resident=True)
        g.cr.enqueue_mode = False
        g.cr.enqueue_mode_async_enable = False
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / steps
        res[key].append(g.flops / ms / 1e9)
    print(f"round {r} done", flush=True)

out = {}
for (m, t), v in res.items():
    g = runs[(m, t)]
    c = g.result(download=True)[:256]
    err = float(abs(c - g.reference(slice(0, 256))).max())
    out[f"{m}x{n}x{k}/{t}/g{gm}"] = {"median_tflops": round(statistics.median(v), 1),
                                    "min_tflops": round(min(v), 1), "max_tflops": round(max(v), 1),
                                    "max_err_rows0_255": err, "handover_fallbacks": g.handover_fallbacks()}
print(json.dumps(out, indent=1))
