"""GPU probe: the headline GEMM (8192³ bf16, device-resident) on async
enqueue queues with Q compute streams in a fresh process: ms per GEMM over
K back-to-back computes (median of rounds), every C tile checked once."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.ops.gemm import GEMM_LIBS, GemmBf16  # noqa: E402
from cekirdekler_amd.ops.library import library  # noqa: E402

Q = int(sys.argv[1]) if len(sys.argv) > 1 else 4
K = 20
gpu = ck.ClPlatforms.all().gpus()[0]
cr = ck.ClNumberCruncher(gpu, "", prebuilt=library(*GEMM_LIBS), queue_concurrency=Q)
g = GemmBf16(8192, 8192, 8192, cruncher=cr, tile="256x256pb")
for _ in range(5):
    g.run(compute_id=1, resident=True)
rounds = {"one_queue": [], "async": []}
for r in range(5):
    for mode in ("one_queue", "async"):
        torch.cuda.synchronize()
        t = time.perf_counter()
        cr.enqueue_mode = True
        cr.enqueue_mode_async_enable = mode == "async"
        for _ in range(K):
            g.run(compute_id=1, resident=True)
        cr.enqueue_mode = False
        cr.enqueue_mode_async_enable = False
        torch.cuda.synchronize()
        rounds[mode].append((time.perf_counter() - t) * 1e3 / K)
err, tiles = g.verify_full(compute_id=1)
print(json.dumps({"Q": Q, **{m: round(statistics.median(v), 4) for m, v in rounds.items()},
                  "max_rel_err_full": err, "tiles_checked": tiles}), flush=True)
cr.dispose()
