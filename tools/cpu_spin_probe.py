"""CPU-device host cost with and without spinning pool threads (run it
under CEK_POOL_SPIN_US=0 and =50): a tiny compute on one and on two CPU
devices, and the wave example's frame on the CPU device.  Timings of the
CPU environment the GPU boxes give a process (a cgroup share of a larger
machine), which the builder's VM does not reproduce.

    python tools/cpu_spin_probe.py [out.json]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.hardware import usable_cpus  # noqa: E402
from cekirdekler_amd.models.wave import WaveSurface, grid_mesh  # noqa: E402

SRC = "__global__ void inc(float* x) { x[get_global_id(0)] += 1.0f; }"


def tiny(ndev, reps=2000):
    cpu = ck.ClPlatforms.all().cpus(True)
    devs = cpu
    for _ in range(ndev - 1):
        devs = devs + cpu
    cr = ck.ClNumberCruncher(devs, SRC)
    n = 4096 * ndev
    x = ck.ClArray(np.zeros(n, np.float32))
    for _ in range(200):
        x.compute(cr, 1, "inc", n, 256)
    t = time.perf_counter()
    for _ in range(reps):
        x.compute(cr, 1, "inc", n, 256)
    us = (time.perf_counter() - t) * 1e6 / reps
    cr.dispose()
    return round(us, 2)


def wave(frames=300):
    base, nrm = grid_mesh(224, 256)
    w = WaveSurface(base, nrm, devices=ck.ClPlatforms.all().cpus(True))
    for _ in range(50):
        w.update()
    t = time.perf_counter()
    for _ in range(frames):
        w.update()
    ms = (time.perf_counter() - t) * 1e3 / frames
    w.cr.dispose()
    return round(ms, 4)


res = {"pool_spin_us": float(os.environ.get("CEK_POOL_SPIN_US", "0")), "usable_cpus": usable_cpus(),
       "cpu_count": os.cpu_count(), "tiny_1dev_us": tiny(1), "tiny_2dev_us": tiny(2), "wave_cpu_ms": wave()}
js = json.dumps(res)
print(js)
if len(sys.argv) > 1:
    with open(sys.argv[1], "w") as f:
        f.write(js + "\n")
