"""GPU probe: PCIe rates of 256 MiB copies between pinned host memory and
the GPU, one direction at a time and both at once (H2D and D2H on two
streams): the floor of any host-resident call that moves A, B up and C down.
"""
import json
import statistics
import time

import torch

nbytes = 256 << 20
d_up = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
d_dn = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
h_up = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
h_dn = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
s_up, s_dn = torch.cuda.Stream(), torch.cuda.Stream()


def run(up: bool, dn: bool) -> float:
    ts = []
    for _ in range(8):
        torch.cuda.synchronize()
        t = time.perf_counter()
        if up:
            with torch.cuda.stream(s_up):
                d_up.copy_(h_up, non_blocking=True)
        if dn:
            with torch.cuda.stream(s_dn):
                h_dn.copy_(d_dn, non_blocking=True)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    return statistics.median(ts)


out = {}
for name, up, dn in (("h2d", True, False), ("d2h", False, True), ("both", True, True)):
    ms = run(up, dn)
    moved = nbytes * (int(up) + int(dn))
    out[name] = {"ms": round(ms, 3), "GBps": round(moved / (ms * 1e-3) / 1e9, 1)}
print(json.dumps(out), flush=True)
