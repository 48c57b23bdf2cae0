"""The CPU device alone three ways on the hetero_stream workload (iters 16):
a CPU-only cruncher with every usable thread, one with 14 threads, and a
GPU+CPU cruncher with its GPU disabled (the configuration the overhead-aware
balancer probes).  Interleaved rounds; median ms per call.

    python tools/mixed_cpu_alone_probe.py
"""
import sys, time, statistics, json
sys.path.insert(0, '.')
import numpy as np
import cekirdekler_amd as ck
SRC = """
__global__ void poly(const float* x, float* y) {
    long long i = get_global_id(0);
    float v = x[i], acc = y[i];
    for (int k = 0; k < 16; ++k) acc = fmaf(acc, v, 0.25f);
    y[i] = acc;
}"""
n = 64 << 20
p = ck.ClPlatforms.all()
x = ck.ClArray(n, np.float32); x.array[:] = 0.5; x.read_only = True; x.partial_read = True
y = ck.ClArray(n, np.float32); y.partial_read = True
cr15 = ck.ClNumberCruncher(p.cpus(True), SRC)
cr14 = ck.ClNumberCruncher(p.cpus(True, max_cpu_cores=14), SRC)
mixed = ck.ClNumberCruncher(p.gpus()[0] + p.cpus(True), SRC)
mixed.disable_device(0)
crs = {"cpu15": cr15, "cpu14": cr14, "mixed_cpu_only": mixed}
def call(cr): x.next_param(y).compute(cr, 1, "poly", n, 256, pipeline=True, pipeline_blobs=8)
for cr in crs.values():
    for _ in range(5): call(cr)
res = {k: [] for k in crs}
for _ in range(5):
    for k, cr in crs.items():
        t = time.perf_counter()
        for _ in range(4): call(cr)
        res[k].append(round((time.perf_counter() - t) * 1e3 / 4, 3))
print(json.dumps({k: (statistics.median(v), v) for k, v in res.items()}))
print("threads", cr15.cores.device(0).cpu_threads, cr14.cores.device(0).cpu_threads, mixed.cores.device(1).cpu_threads)
