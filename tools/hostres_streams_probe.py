"""Host-resident SGEMM 8192³ through compute() (square shells, 16 panels):
stream layouts A/B.  The shell stream is the event
pipeline: uploads on the main stream, kernels on two half-pipeline streams,
downloads on two write streams (5 streams), or on ONE write stream (4
streams, one per hardware queue).  The cruncher's async queue count (4 = the
hardware queues, the new default, vs the reference's 16) is crossed with it
although the event pipeline does not use those queues.  Rounds interleaved,
every C tile checked.

    python tools/hostres_streams_probe.py [rounds] > gpurun_out/hostres_streams.json
"""
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

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
gpu = ck.ClPlatforms.all().gpus()[0]
S = 8192
configs = {}
for q in (4, 16):
    cr = ck.ClNumberCruncher(gpu, "", prebuilt=library(*GEMM_LIBS), queue_concurrency=q)
    g = GemmBf16(S, S, S, cruncher=cr, tile="256x256pb")
    for one in (False, True):
        configs[f"q{q}_{'4streams' if one else '5streams'}"] = (cr, g, one)
times = {k: [] for k in configs}
errs = {}
for name, (cr, g, one) in configs.items():
    cr.cores.pipeline_writes_one_stream = one
    g.run_shells(16, compute_id=3)
    g.run_shells(16, compute_id=3)
    torch.cuda.synchronize()
    errs[name] = g.verify_full(compute_id=3, host=True)
for _ in range(rounds):
    for name, (cr, g, one) in configs.items():
        cr.cores.pipeline_writes_one_stream = one
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            g.run_shells(16, compute_id=3)
        torch.cuda.synchronize()
        times[name].append((time.perf_counter() - t0) * 1e3 / 3)
print(json.dumps({"rounds": rounds, "ms": {k: round(statistics.median(v), 3) for k, v in times.items()},
                  "ms_runs": {k: [round(x, 3) for x in v] for k, v in times.items()},
                  "max_rel_err_full": {k: v[0] for k, v in errs.items()},
                  "tiles_checked": {k: v[1] for k, v in errs.items()}}), flush=True)
