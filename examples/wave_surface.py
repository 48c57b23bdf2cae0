"""The reference's Unity example (Kamera.cs): a wave on 57,344 mesh vertices,
computed on the GPU plus the CPU device with the load balancer splitting the
vertices, versus the CPU device alone ("CPU+GPU 3x as fast", Kamera.cs:266)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import time

import cekirdekler_amd as ck
from cekirdekler_amd.models.wave import WaveSurface, grid_mesh

base, normals = grid_mesh(224, 256)
plats = ck.ClPlatforms.all()
configs = {"cpu": plats.cpus(True)}
if len(plats.gpus()):
    configs["gpu+cpu"] = plats.gpus()[0] + plats.cpus(True)
for name, devs in configs.items():
    w = WaveSurface(base, normals, devices=devs)
    for _ in range(20):
        w.update()
    t = time.perf_counter()
    for _ in range(200):
        w.update()
    ms = (time.perf_counter() - t) / 200 * 1e3
    print(f"{name:8s} {ms:7.3f} ms/frame  split={w.cr.ranges(1)}")
    w.cr.dispose()
