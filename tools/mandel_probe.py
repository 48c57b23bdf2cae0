#!/usr/bin/env python3
"""Mandelbrot 4096² kernel variants on one GPU: kernel-only time (image left
in device memory), useful TFLOP/s (8 FLOP per executed escape iteration) and
agreement with the "quad" kernel.  Optional extra code objects built on the
box: ``--extra path|kernel,ppw`` (e.g. a -fno-slp-vectorize build)."""
import argparse
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.models import mandelbrot as mb  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=4096)
ap.add_argument("--iters", type=int, default=256)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--extra", action="append", default=[])
ap.add_argument("--only", default="", help="comma-separated kernel keys (default: all)")
a = ap.parse_args()
g0 = ck.ClPlatforms.all().gpus()[0]

variants = [(k, None) for k in mb.KERNELS if not a.only or k in a.only.split(",")]
for e in a.extra:
    path, rest = e.split("|")
    name, ppw = rest.split(",")
    key = f"{name}@{path.rsplit('/', 1)[-1]}"
    mb.KERNELS[key] = (name, int(ppw), 256)
    variants.append((key, path + "|" + name))

ref_img = None
for key, prebuilt in variants:
    cr = ck.ClNumberCruncher(g0, "", prebuilt=prebuilt) if prebuilt else None
    m = mb.MandelbrotRenderer(a.size, a.size, a.iters, devices=g0, kernel=key, cruncher=cr)
    img = m.render(1, pipeline=False).copy()
    flops = m.flops()
    if ref_img is None:
        ref_img = img
    mism = int((img != ref_img).sum())
    m.out.write = False
    m.view.read = m.size.read = False
    for _ in range(3):
        m.render(2, pipeline=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        m.render(2, pipeline=False)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.reps * 1e3
    print(json.dumps({"variant": key, "kernel_ms": round(ms, 4), "useful_tflops": round(flops / ms / 1e9, 2),
                      "pct_fp32_peak": round(flops / ms / 1e9 / 157.3 * 100, 1),
                      "mismatch_vs_quad": mism}), flush=True)
    m.cr.dispose()
