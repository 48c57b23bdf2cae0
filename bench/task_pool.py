"""BASELINE config 5: a task pool of 256 mixed non-separable kernels,
greedy asynchronous schedule over a device pool (all GPUs; with one GPU the
same GPU is added several times, as the reference allows).  Reports makespan
against the ideal Σ(task time)/GPUs, where a task's time is its kernel's
device time (hipEvent span from ``record_timeline``, one task at a time on
one GPU) — host launch and sync overheads are not in the ideal, and the
excess is the scheduler's overhead plus imbalance (BASELINE target ≤ 1.15).
The ideal is not a strict floor: with several tasks in flight on one GPU
(3 queues per device) one kernel's tail work-groups run beside the next
kernel's, which the serial spans cannot do, so a well-packed pool can land
slightly under 1 (0.99 measured on one MI355X)."""
import argparse
import time

import numpy as np

from common import emit, sync

import cekirdekler_amd as ck
from cekirdekler_amd.parallel.pool import ClDevicePool, ClDevicePoolType, ClTaskPool

SRC = r"""
__global__ void spin(float* x, const int* it) {
  long long i = get_global_id(0);
  float v = x[i];
  int n = it[0];
  for (int k = 0; k < n; ++k) v = v * 0.9999f + 0.5f;
  x[i] = v;
}
__global__ void saxpy(float* x, const int* it) {
  long long i = get_global_id(0);
  x[i] = 2.0f * x[i] + (float)it[0];
}
"""

ap = argparse.ArgumentParser()
ap.add_argument("--tasks", type=int, default=256)
ap.add_argument("--gpus", type=int, default=0)
ap.add_argument("--logical", type=int, default=2, help="logical devices per GPU when only one GPU")
ap.add_argument("--queues", type=int, default=3)
a = ap.parse_args()
g = ck.ClPlatforms.all().gpus()
ng = len(g) if a.gpus <= 0 else min(a.gpus, len(g))
devs = g[0:ng]
if ng == 1 and a.logical > 1:
    for _ in range(a.logical - 1):
        devs = devs + g[0]
rng = np.random.default_rng(3)
N = 1 << 22
tasks = []
for t in range(a.tasks):
    kind = "spin" if t % 4 else "saxpy"
    iters = int(rng.choice([256, 512, 1024, 2048]))
    x = ck.ClArray(np.ones(N, np.float32))
    x.read = x.write = False
    it = ck.ClArray(np.array([iters], np.int32))
    it.write = False
    tasks.append((kind, x, it))

# per-task device times, serially on one device (hipEvent-timed kernel spans)
ref_cr = ck.ClNumberCruncher(g[0], SRC)
for kind, x, it in tasks:
    x.next_param(it).compute(ref_cr, 1, kind, N, 256)
sync()
ref_cr.record_timeline = True
for kind, x, it in tasks:
    x.next_param(it).compute(ref_cr, 1, kind, N, 256)
single = [sp["end_ms"] - sp["begin_ms"] for sp in ref_cr.timeline()]
assert len(single) == len(tasks), (len(single), len(tasks))
ref_cr.dispose()

pool = ClDevicePool(ClDevicePoolType.DEVICE_COMPUTE_AT_WILL, SRC, True, a.queues)
pool.add_device(devs)
tp = ClTaskPool()
for kind, x, it in tasks:
    tp.feed(x.next_param(it).task(1, kind, N, 256))
# warm the pool's crunchers/buffers once
pool.enqueue_task_pool(tp)
pool.finish()
for kind, x, it in tasks:
    tp.feed(x.next_param(it).task(1, kind, N, 256))
sync()
t = time.perf_counter()
pool.enqueue_task_pool(tp)
pool.finish()
sync()
makespan = (time.perf_counter() - t) * 1e3
ideal = sum(single) / max(1, ng)
emit({"config": "task_pool_256", "tasks": a.tasks, "gpus": ng, "logical_devices": len(devs),
      "makespan_ms": makespan, "ideal_ms_sum_over_gpus": ideal, "ideal_basis": "hipEvent device time per task", "makespan_over_ideal": makespan / ideal,
      "tasks_per_s": a.tasks / (makespan * 1e-3), "per_device_tasks": pool.device_task_counts()})
pool.dispose()
