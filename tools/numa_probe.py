"""Host NUMA placement of the CPU device: does it explain the spread of
GPU+CPU splits between crunchers on one box?

Prints the node → CPU map and each GPU's node, then for each placement
(threads floating over every CPU; the threads and the arrays' first touch
bound to one node) times the CPU device alone and GPU+CPU by the law on the
hetero_stream workload (host-resident x, y; y = y·x + 0.25).  Pool threads
inherit the creating thread's affinity, so binding the calling thread before
the cruncher is built binds its pool.

    python tools/numa_probe.py [--n 67108864] [--calls 30]
"""
import argparse
import glob
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import cekirdekler_amd as ck  # noqa: E402

SRC = """
__global__ void poly(const float* x, float* y) {
    long long i = get_global_id(0);
    y[i] = fmaf(y[i], x[i], 0.25f);
}
"""

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=64 << 20)
ap.add_argument("--calls", type=int, default=30)
ap.add_argument("--out", default="gpurun_out/numa_probe.json")
a = ap.parse_args()


def cpulist(s):
    out = []
    for part in s.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        out += list(range(int(lo), int(hi or lo) + 1))
    return out


nodes = {}
for d in sorted(glob.glob("/sys/devices/system/node/node[0-9]*")):
    nodes[int(d.rsplit("node", 1)[1])] = cpulist(open(d + "/cpulist").read())
gpu_nodes = []
for d in sorted(glob.glob("/sys/class/drm/card[0-9]*/device/numa_node")):
    try:
        gpu_nodes.append(int(open(d).read()))
    except (OSError, ValueError):
        pass
full = sorted(os.sched_getaffinity(0))
res = {"nodes": {k: [v[0], v[-1], len(v)] for k, v in nodes.items()}, "gpu_nodes": gpu_nodes,
       "affinity_cpus": len(full), "usable_cpus": ck.hardware.usable_cpus()}
print(json.dumps(res), flush=True)

plats = ck.ClPlatforms.all()
gpu = plats.gpus()
node_of_gpu0 = None
try:
    info = gpu.device(0).native_info()
    p = glob.glob(f"/sys/bus/pci/devices/*:{info.pci_bus:02x}:{info.pci_device:02x}.0/numa_node")
    res["gpu0_pci"] = [info.pci_bus, info.pci_device, p[:1]]
    node_of_gpu0 = int(open(p[0]).read()) if p else None
except Exception as e:  # noqa: BLE001
    res["gpu0_node_error"] = str(e)
res["gpu0_node"] = node_of_gpu0

placements = [("float", None)]
for k in sorted(nodes)[:2]:
    placements.append((f"node{k}", nodes[k][:16]))


def timed(cr, x, y, calls):
    def call():
        x.next_param(y).compute(cr, 1, "poly", a.n, 256, pipeline=True, pipeline_blobs=8)
    for _ in range(calls):
        call()
    ts = []
    for _ in range(calls):
        t = time.perf_counter()
        call()
        ts.append((time.perf_counter() - t) * 1e3)
    return statistics.median(ts)


for name, cpus in placements:
    if cpus is not None:
        os.sched_setaffinity(0, cpus)
    try:
        x = ck.ClArray(a.n, np.float32)
        x.array[:] = 0.5
        x.read_only = True
        x.partial_read = True
        y = ck.ClArray(a.n, np.float32)
        y.array[:] = 0.25
        y.partial_read = True
        cpu = plats.cpus(True)
        r = {}
        cr = ck.ClNumberCruncher(cpu, SRC)
        r["cpu_ms"] = timed(cr, x, y, a.calls)
        cr.dispose()
        if len(gpu):
            cr = ck.ClNumberCruncher(gpu[0] + cpu, SRC)
            r["gpu+cpu_ms"] = timed(cr, x, y, a.calls)
            rr = cr.ranges(1)
            r["gpu_share"] = rr[0] / sum(rr)
            rec = cr.last_record()
            r["device_ms"] = [round(v, 3) for v in rec["device_ms"]]
            cr.dispose()
        res[name] = r
        print(name, json.dumps(r), flush=True)
        del x, y
    finally:
        os.sched_setaffinity(0, full)

os.makedirs(os.path.dirname(a.out), exist_ok=True)
json.dump(res, open(a.out, "w"))
