"""Greedy task scheduling (reference ClTaskPool / ClDevicePool): independent
kernels are taken by whichever device is free; callbacks fire on completion."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np

import cekirdekler_amd as ck
from cekirdekler_amd.parallel.pool import ClDevicePool, ClDevicePoolType, ClTaskPool

SRC = """__global__ void work(float* x, float* v) {
    long long i = get_global_id(0); float s = x[i];
    for (int k = 0; k < 256; ++k) s = s * 0.999f + v[0];
    x[i] = s; }"""
plats = ck.ClPlatforms.all()
devs = (plats.gpus()[0] + plats.gpus()[0]) if len(plats.gpus()) else (plats.cpus(True) + plats.cpus(True))
pool = ClDevicePool(ClDevicePoolType.DEVICE_COMPUTE_AT_WILL, SRC, True, 8)
pool.add_device(devs)
tasks = ClTaskPool()
done = []
for i in range(64):
    x = ck.ClArray(np.zeros(1 << 16, np.float32))
    v = ck.ClArray(np.array([float(i)], np.float32)); v.write = False
    t = x.next_param(v).task(1, "work", 1 << 16, 256)
    t.set_callback(lambda i=i: done.append(i))
    tasks.feed(t)
pool.enqueue_task_pool(tasks)
pool.finish()
print("tasks per device:", pool.device_task_counts(), "callbacks:", len(done))
pool.dispose()
