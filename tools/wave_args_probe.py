"""GPU probe: the wave example's GPU-only frame (57,344 vertices, one
synchronous compute() per frame, displaced vertices written zero-copy) with
the 256-byte argument block uploaded by a copy every frame (the default)
against the kernel reading it straight from pinned host memory
(``arguments.zero_copy``: no copy command in the frame's stream).  Frame
time (median of interleaved rounds), the kernel's own time (dispatch
timestamps) and the output against the numpy reference.

    python tools/wave_args_probe.py [rounds] [frames]
"""
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.models.wave import WaveSurface, grid_mesh  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 200
gpu = ck.ClPlatforms.all().gpus()[0]
base, normals = grid_mesh(224, 256)
cfg = {}
for zc_args in (False, True):
    w = WaveSurface(base, normals, devices=gpu)
    w.arguments.zero_copy = zc_args
    for _ in range(100):
        w.update()
    cfg["args_zc" if zc_args else "args_copy"] = w
runs = {k: [] for k in cfg}
compute_only = {k: [] for k in cfg}
for _ in range(rounds):
    for k, w in cfg.items():
        t = time.perf_counter()
        for _ in range(frames):
            w.update()
        runs[k].append((time.perf_counter() - t) * 1e3 / frames)
out = {}
for k, w in cfg.items():
    w.cr.record_kernel_times = True
    for _ in range(50):
        w.update()
    w.cr.record_kernel_times = False
    kt = sorted(ms for name, ms in w.cr.kernel_times(0) if name.startswith("waveEquation"))
    err = float(np.abs(w.update()["z"] - w.reference()["z"]).max())
    out[k] = {"ms_per_frame": round(statistics.median(runs[k]), 4),
              "ms_rounds": [round(x, 4) for x in runs[k]],
              "kernel_ms_median": round(kt[len(kt) // 2], 4) if kt else None,
              "max_abs_err": err, "record": {x: w.cr.last_record().get(x) for x in ("h2d_bytes", "d2h_bytes")}}
for w in cfg.values():
    w.cr.dispose()
print(json.dumps(out), flush=True)
