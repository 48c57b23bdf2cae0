"""Host-resident SGEMM 8192³ calls for a copy/kernel trace: the square-shell
stream through compute() (the bench's host-resident mode) and the native
shell entry point, a few calls each, with wall times.  Run it under
``rocprofv3 --kernel-trace --memory-copy-trace`` to see when every upload,
kernel and download of a call ran.

    python tools/hostres_probe.py [panels,...] [calls]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.ops.gemm import GEMM_LIBS, GemmBf16  # noqa: E402
from cekirdekler_amd.ops.library import library  # noqa: E402

panel_list = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "16").split(",")]
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 4
cr = ck.ClNumberCruncher(ck.ClPlatforms.all().gpus()[0], "", prebuilt=library(*GEMM_LIBS))
g = GemmBf16(8192, 8192, 8192, cruncher=cr, tile="256x256pb")
out = {"panels": panel_list}
runs = [(f"compute_shells_p{p}", (lambda p=p, i=i: g.run_shells(p, compute_id=3 + i)))
        for i, p in enumerate(panel_list)]
# the last shells split into R_s / C_s blobs (16 panels)
runs += [(f"compute_shells_p16_split{k}", (lambda k=k: g.run_shells(16, compute_id=20 + k, split_last=k)))
         for k in (2, 4, 8)]
runs.append((f"native_shells_p{panel_list[0]}", lambda: g.run_host_shells(panel_list[0])))
for name, fn in runs:
    fn()
    torch.cuda.synchronize()
    ms = []
    for _ in range(calls):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ms.append(round((time.perf_counter() - t) * 1e3, 3))
    out[name + "_ms"] = ms
print(json.dumps(out))
cr.dispose()
