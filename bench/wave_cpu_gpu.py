"""The reference's only published speed claim, measured: the Unity wave
example on 224×256 = 57,344 vertices, local 64, "3× as fast" with CPU+GPU
than CPU-only (Kamera.cs:266, devices from devicesAmd(true, true)).

Frames per second of WaveSurface.update() (one compute per frame, the
displaced vertices downloaded every frame, as the Unity loop uses them) on
the CPU device alone, the GPU alone, and GPU + CPU with the load balancer
splitting the vertices.  Steady state after the balancer has converged.
``reference_cpu`` is the denominator of the reference's own claim: its
CPU-only strategy, a single-threaded scalar loop with no runtime
(Kamera.cs:208-218, ``ReferenceCpuWave``); ``cpu`` is this framework's
multi-threaded, vectorised CPU device.
``gpu+cpu_fit`` is the same pair with the opt-in overhead-aware balancer
(``overhead_aware_balancer``: t = a + b·range per device), which may leave
the CPU out when its share does not pay for the second device's fixed cost."""
import argparse
import statistics
import time

import numpy as np

from common import emit

import cekirdekler_amd as ck
from cekirdekler_amd.models.wave import ReferenceCpuWave, WaveSurface, grid_mesh

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=200)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--nx", type=int, default=224)
ap.add_argument("--ny", type=int, default=256)
a = ap.parse_args()
plats = ck.ClPlatforms.all()
cpu, gpus = plats.cpus(True), plats.gpus()
base, normals = grid_mesh(a.nx, a.ny)
configs = [("cpu", cpu)]
if len(gpus):
    configs += [("gpu", gpus[0]), ("gpu+cpu", gpus[0] + cpu), ("gpu+cpu_fit", gpus[0] + cpu)]
out = {"config": "wave_cpu_gpu", "vertices": len(base), "local": 64,
       "timing": f"median of {a.rounds} interleaved rounds of {a.frames // a.rounds} frames per config"}
surfaces = {"reference_cpu": ReferenceCpuWave(base, normals)}
for _ in range(10):
    surfaces["reference_cpu"].update()
for name, devs in configs:
    w = WaveSurface(base, normals, devices=devs)
    if name.endswith("_fit"):
        w.cr.overhead_aware_balancer = True
    for _ in range(100):  # balancer (and the predictor's probe) converge, buffers resident
        w.update()
    surfaces[name] = w
# the configs take turns (a round of frames each), so clock and host-load
# drift over the run hits every config alike
per = max(1, a.frames // a.rounds)
runs = {name: [] for name in surfaces}
for _ in range(a.rounds):
    for name, w in surfaces.items():
        t = time.perf_counter()
        for _ in range(per):
            w.update()
        runs[name].append((time.perf_counter() - t) * 1e3 / per)
for name, w in surfaces.items():
    out[f"{name}_ms_per_frame"] = statistics.median(runs[name])
    out[f"{name}_ms_rounds"] = [round(x, 4) for x in runs[name]]
    out[f"{name}_max_abs_err"] = float(np.abs(w.update()["z"] - w.reference()["z"]).max())
    if name == "reference_cpu":
        continue
    if name.startswith("gpu+cpu"):
        out[f"{name}_shares"] = [r / sum(w.cr.ranges(1)) for r in w.cr.ranges(1)]
    if name.endswith("_fit"):
        out[f"{name}_predictor"] = {k: v for k, v in w.cr.balancer_predictor_info(1).items()}
for w in surfaces.values():
    if hasattr(w, "cr"):
        w.cr.dispose()
ref = out["reference_cpu_ms_per_frame"]
out["speedup_cpu_device_over_reference_cpu"] = ref / out["cpu_ms_per_frame"]
if "gpu+cpu_ms_per_frame" in out:
    out["speedup_gpu+cpu_over_cpu"] = out["cpu_ms_per_frame"] / out["gpu+cpu_ms_per_frame"]
    out["speedup_gpu_over_cpu"] = out["cpu_ms_per_frame"] / out["gpu_ms_per_frame"]
    out["speedup_gpu+cpu_fit_over_cpu"] = out["cpu_ms_per_frame"] / out["gpu+cpu_fit_ms_per_frame"]
    out["speedup_gpu_over_reference_cpu"] = ref / out["gpu_ms_per_frame"]
    out["speedup_gpu+cpu_over_reference_cpu"] = ref / out["gpu+cpu_ms_per_frame"]
    out["speedup_gpu+cpu_fit_over_reference_cpu"] = ref / out["gpu+cpu_fit_ms_per_frame"]
    out["fit_not_slower_than_gpu_alone"] = out["gpu+cpu_fit_ms_per_frame"] <= 1.02 * out["gpu_ms_per_frame"]
emit(out)
