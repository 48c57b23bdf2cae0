"""GPU probe: N-body force+integrate throughput through compute()."""
import json
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.models.nbody import NBodySimulation  # noqa: E402

g0 = ck.ClPlatforms.all().gpus()[0]
res = {}
for n in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "65536,262144").split(",")]:
    sim = NBodySimulation(n, devices=g0)
    sim.step()
    torch.cuda.synchronize()
    reps = max(2, int(2e10 // (n * n)))
    t = time.perf_counter()
    for _ in range(reps):
        sim.step()
    torch.cuda.synchronize()
    s = (time.perf_counter() - t) / reps
    res[n] = {"ms": s * 1e3, "ginter_per_s": n * n / s / 1e9, "tflops_20": 20 * n * n / s / 1e12}
print(json.dumps(res, indent=1))
