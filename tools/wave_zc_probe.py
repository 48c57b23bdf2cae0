"""GPU probe: the wave example's GPU-only frame (57,344 vertices, one
synchronous compute() per frame) with the 256-byte argument block in a
pinned (hipHostMalloc) array instead of wrapped numpy memory, and with the
displaced vertices written zero-copy (the kernel stores straight into the
registered host array; no D2H).  Configs interleaved over rounds, median
ms per frame, outputs checked against the numpy reference.

    python tools/wave_zc_probe.py [rounds] [frames]
"""
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.arrays import ClArray  # noqa: E402
from cekirdekler_amd.models.wave import WaveSurface, grid_mesh  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 200
gpu = ck.ClPlatforms.all().gpus()[0]
base, normals = grid_mesh(224, 256)


def make(pinned_args: bool, zc_out: bool) -> WaveSurface:
    w = WaveSurface(base, normals, devices=gpu, zero_copy_output=zc_out)
    if not pinned_args:  # the round-3 layout: wrapped (pageable) numpy memory
        a = ClArray(np.zeros(64, np.float32))
        a.write = False
        a.partial_read = False
        w.arguments = a
    for _ in range(100):
        w.update()
    return w


cfg = {"base": make(False, False), "pinned_args": make(True, False), "pinned_args+zc_out": make(True, True)}
runs = {k: [] for k in cfg}
for _ in range(rounds):
    for k, w in cfg.items():
        t = time.perf_counter()
        for _ in range(frames):
            w.update()
        runs[k].append((time.perf_counter() - t) * 1e3 / frames)
out = {}
for k, w in cfg.items():
    err = float(np.abs(w.update()["z"] - w.reference()["z"]).max())
    out[k] = {"ms_per_frame": round(statistics.median(runs[k]), 4), "max_abs_err": err}
    w.cr.dispose()
print(json.dumps(out))
