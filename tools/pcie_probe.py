"""GPU probe: PCIe copy rates (pinned host memory) for one 64 MiB copy split
over 1, 2 or 4 concurrent streams, both directions, and the Mandelbrot
4096² end-to-end render at several blob counts of the event and driver
pipelines."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

out = {}
nbytes = 64 << 20
dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
for nstreams in (1, 2, 4):
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    chunk = nbytes // nstreams
    for name, fn in (("d2h", lambda d, h: h.copy_(d, non_blocking=True)),
                     ("h2d", lambda d, h: d.copy_(h, non_blocking=True))):
        ts = []
        for rep in range(12):
            torch.cuda.synchronize()
            t = time.perf_counter()
            for i, s in enumerate(streams):
                with torch.cuda.stream(s):
                    fn(dev[i * chunk:(i + 1) * chunk], host[i * chunk:(i + 1) * chunk])
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        best = sorted(ts[2:])[len(ts[2:]) // 2]
        out[f"{name}_{nstreams}streams"] = {"ms": best * 1e3, "GBps": nbytes / best / 1e9}
# both directions at once (full duplex)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
dev2 = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
host2 = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
ts = []
for rep in range(12):
    torch.cuda.synchronize()
    t = time.perf_counter()
    with torch.cuda.stream(s1):
        host.copy_(dev, non_blocking=True)
    with torch.cuda.stream(s2):
        dev2.copy_(host2, non_blocking=True)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t)
best = sorted(ts[2:])[len(ts[2:]) // 2]
out["duplex_64MiB_each_way"] = {"ms": best * 1e3, "GBps_per_direction": nbytes / best / 1e9}
print(json.dumps(out), flush=True)

import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.models.mandelbrot import MandelbrotRenderer  # noqa: E402

m = MandelbrotRenderer(4096, 4096, 256, devices=ck.ClPlatforms.all().gpus()[0])
res = {}
for ptype, pname in ((True, "event"), (False, "driver")):
    for blobs in (4, 8, 16, 32):
        cid = 100 + blobs + (0 if ptype else 1000)
        for _ in range(3):
            m.render(cid, pipeline=True, blobs=blobs, pipeline_type=ptype)
        torch.cuda.synchronize()
        ts = []
        for _ in range(15):
            t = time.perf_counter()
            m.render(cid, pipeline=True, blobs=blobs, pipeline_type=ptype)
            ts.append((time.perf_counter() - t) * 1e3)
        res[f"{pname}_b{blobs}"] = round(sorted(ts)[len(ts) // 2], 4)
print(json.dumps({"mandelbrot_e2e_ms_median": res}), flush=True)
