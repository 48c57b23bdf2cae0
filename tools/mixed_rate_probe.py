"""The CPU device's rate inside a GPU+CPU cruncher against a CPU-only cruncher
of the same thread count (the measurement of
tests/test_gpu_features.py::test_cpu_device_inside_gpu_cpu_cruncher_keeps_its_speed),
with the mixed call's GPU time and the process's CPU time per call.

    python tools/mixed_rate_probe.py [--samples 40]      (one setting per process;
    set CEK_MIXED_CPU / CEK_HIP_SYNC / CEK_ADAPTIVE_SLEEP in the environment)
"""
import argparse
import json
import os
import resource
import statistics
import sys

import numpy as np

sys.path.insert(0, ".")
import cekirdekler_amd as ck  # noqa: E402

SRC = r"""
__global__ void poly(const float* x, float* y) {
    long long i = get_global_id(0);
    float v = x[i], acc = 1.0f;
    for (int k = 0; k < 96; ++k) acc = fmaf(acc, v, 0.25f);
    y[i] = acc;
}"""

ap = argparse.ArgumentParser()
ap.add_argument("--samples", type=int, default=40)
ap.add_argument("--n", type=int, default=1 << 22)
a = ap.parse_args()


def cpu_ms():
    r = resource.getrusage(resource.RUSAGE_SELF)
    return (r.ru_utime + r.ru_stime) * 1e3


p = ck.ClPlatforms.all()
mixed = ck.ClNumberCruncher(p.gpus()[0] + p.cpus(True), SRC)
threads = mixed.cores.device(1).cpu_threads
n = a.n
x = ck.ClArray(np.random.default_rng(0).uniform(0.1, 0.9, n).astype(np.float32))
y = ck.ClArray(np.zeros(n, np.float32))
x.write = False
y.read = False
for _ in range(20):
    x.next_param(y).compute(mixed, 1, "poly", n, 256)
r_cpu = (mixed.ranges(1)[1] // 256) * 256
alone = ck.ClNumberCruncher(p.cpus(True, max_cpu_cores=threads), SRC)
xs = ck.ClArray(x.array[:r_cpu].copy())
ys = ck.ClArray(np.zeros(r_cpu, np.float32))
xs.write = False
ys.read = False
xs.next_param(ys).compute(alone, 1, "poly", r_cpu, 256)
m_rate, a_rate, gpu_ms, m_cpu, a_cpu, m_wall, a_wall = [], [], [], [], [], [], []
for _ in range(a.samples):
    c0 = cpu_ms()
    x.next_param(y).compute(mixed, 1, "poly", n, 256)
    c1 = cpu_ms()
    rec = mixed.last_record()
    m_rate.append(rec["ranges"][1] / rec["device_ms"][1])
    gpu_ms.append(rec["device_ms"][0])
    m_wall.append(rec["wall_ms"])
    m_cpu.append(c1 - c0)
    xs.next_param(ys).compute(alone, 1, "poly", r_cpu, 256)
    c2 = cpu_ms()
    ra = alone.last_record()
    a_rate.append(r_cpu / ra["device_ms"][0])
    a_wall.append(ra["wall_ms"])
    a_cpu.append(c2 - c1)
med = statistics.median
out = {"env": {k: os.environ.get(k, "") for k in ("CEK_MIXED_CPU", "CEK_HIP_SYNC", "CEK_ADAPTIVE_SLEEP",
                                                   "CEK_SHARED_CPU_POOL")},
       "threads": threads, "r_cpu": r_cpu, "mixed_over_alone": med(m_rate) / med(a_rate),
       "mixed_rate": med(m_rate), "alone_rate": med(a_rate), "mixed_gpu_ms": med(gpu_ms),
       "mixed_wall_ms": med(m_wall), "alone_wall_ms": med(a_wall),
       "mixed_process_cpu_ms_per_call": med(m_cpu), "alone_process_cpu_ms_per_call": med(a_cpu),
       "same_pool": mixed._cores.cpu_pool_id(1) == alone._cores.cpu_pool_id(0)}
print(json.dumps(out), flush=True)
mixed.dispose()
alone.dispose()
