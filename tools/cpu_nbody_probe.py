"""CPU-device throughput of the tester's n-body string kernel (Tester.cs's
nBody, utils/tester.nbody): ms per step and interactions/s on the process's
CPU share, checked against float64, with the CPU JIT's runner
(kernel force-inlined into an ``omp simd`` work-item loop)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.hardware import usable_cpus  # noqa: E402
from cekirdekler_amd.utils import tester  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
cpu = ck.ClPlatforms.all().cpus(True)
t = []
rc = tester.nbody(n, cpu, log=False, iterations=5, timing=t)
ms = t[0] / 5
print(json.dumps({"config": "cpu_nbody_string_kernel", "n": n, "threads": usable_cpus(), "ms_per_step": ms,
                  "interactions_per_s": n * n / ms * 1e3, "check_ok": rc == 0}))
