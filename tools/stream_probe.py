"""GPU probe: HBM-bound library kernels through compute() on device-resident
arrays (enqueue mode, interleaved rounds): copy, SAXPY, vector add and the
two reduction kernels.  Reports effective GB/s of bytes moved.

    python tools/stream_probe.py [MiB per array] [rounds] [steps]
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.ops.library import library  # noqa: E402

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
n = mib * 1024 * 1024 // 4
cr = ck.ClNumberCruncher(ck.ClPlatforms.all().gpus()[0], "", prebuilt=library("stream", "reduce"))
x = ck.ClArray(np.random.default_rng(0).random(n, dtype=np.float32))
y = ck.ClArray(np.ones(n, np.float32))
z = ck.ClArray(n, np.float32)
a = ck.ClArray(np.array([0.5], np.float32))
p8 = ck.ClArray(n // 2048, np.float32)
p32 = ck.ClArray(n // 8192, np.float32)
for arr in (x, y, z, a):
    arr.elements_per_work_item = 4
a.elements_per_work_item = 1
p8.elements_per_group = 1
p32.elements_per_group = 1


def flags(first):
    for arr in (x, y, a):
        arr.read = first
        arr.write = False
    for arr in (z, p8, p32):
        arr.read = False
        arr.write = False


cases = {
    # name: (arrays, kernel, global range, local, bytes moved)
    "copy": (lambda: x.next_param(z), "cek_copy_u8", n // 4, 256, 2 * 4 * n),
    "saxpy": (lambda: a.next_param(x, y), "cek_saxpy_f32", n // 4, 256, 3 * 4 * n),
    "vec_add": (lambda: x.next_param(y, z), "cek_vec_add_f32", n // 4, 256, 3 * 4 * n),
    "reduce_x8": (lambda: x.next_param(p8), "cek_reduce_sum_f32", n // 8, 256, 4 * n),
    "reduce_x32": (lambda: x.next_param(p32), "cek_reduce_sum_f32_x32", n // 32, 256, 4 * n),
}
flags(True)
for name, (grp, k, G, L, _) in cases.items():
    if name.startswith("reduce"):
        x.elements_per_work_item = 8 if name == "reduce_x8" else 32
    else:
        x.elements_per_work_item = 4
    grp().compute(cr, 1 + list(cases).index(name), k, G, L)
flags(False)
torch.cuda.synchronize()
res = {k: [] for k in cases}
for _ in range(rounds):
    for i, (name, (grp, k, G, L, nbytes)) in enumerate(cases.items()):
        x.elements_per_work_item = 8 if name == "reduce_x8" else 32 if name == "reduce_x32" else 4
        cr.enqueue_mode = True
        t0 = time.perf_counter()
        for _ in range(steps):
            grp().compute(cr, 1 + i, k, G, L)
        cr.enqueue_mode = False
        torch.cuda.synchronize()
        res[name].append(nbytes / ((time.perf_counter() - t0) / steps) / 1e9)
out = {k: {"median_GBps": round(statistics.median(v), 1), "max_GBps": round(max(v), 1)} for k, v in res.items()}
cr.download(p32, 0)
cr.download(p8, 0)
ref = float(x.array.astype(np.float64).sum())
out["reduce_x8"]["rel_err"] = abs(float(p8.array.astype(np.float64).sum()) - ref) / ref
out["reduce_x32"]["rel_err"] = abs(float(p32.array.astype(np.float64).sum()) - ref) / ref
t = torch.from_numpy(x.array).cuda()
for _ in range(3):
    t.sum()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    t.sum()
torch.cuda.synchronize()
out["torch_sum"] = {"GBps": round(4 * n / ((time.perf_counter() - t0) / steps) / 1e9, 1)}
print(json.dumps({"MiB_per_array": mib, **out}, indent=1))
