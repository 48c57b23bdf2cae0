"""GPU probe: per-frame time of the wave example (GPU only, synchronous
compute() per frame) with the HIP runtime's default host wait and with
hipDeviceScheduleSpin / hipDeviceScheduleYield / hipDeviceScheduleBlockingSync set before any
device work (one process per setting).

    python tools/sched_probe.py [default|spin|yield|block] [frames]
"""
import ctypes
import json
import os
import sys
import time

mode = sys.argv[1] if len(sys.argv) > 1 else "default"
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 400
flags = {"default": None, "spin": 1, "yield": 2, "block": 4}[mode]
if flags is not None:
    hip = ctypes.CDLL("libamdhip64.so")
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(flags))
    print(f"hipSetDeviceFlags({flags}) -> {rc}", flush=True)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.models.wave import WaveSurface, grid_mesh  # noqa: E402

base, nrm = grid_mesh(224, 256)
w = WaveSurface(base, nrm, devices=ck.ClPlatforms.all().gpus()[0])
for _ in range(50):
    w.update()
ts = []
for _ in range(5):
    t = time.perf_counter()
    for _ in range(frames):
        w.update()
    ts.append((time.perf_counter() - t) * 1e3 / frames)
print(json.dumps({"mode": mode, "ms_per_frame": sorted(ts)[2], "runs": [round(x, 4) for x in ts]}), flush=True)
