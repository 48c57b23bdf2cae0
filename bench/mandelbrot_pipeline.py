"""BASELINE config 2: Mandelbrot 4096×4096 on 1×MI355X with the event-driven
read/compute/write pipeline.  Reports end-to-end time (kernels + D2H of the
64 MiB image) for no pipeline / event pipeline / driver pipeline, the
kernel-only time (image left in device memory), and the D2H bound."""
import argparse

import numpy as np

from common import FP32_PEAK_TFLOPS, emit, timeit

import cekirdekler_amd as ck
from cekirdekler_amd.models.mandelbrot import MandelbrotRenderer

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=4096)
ap.add_argument("--iters", type=int, default=256)
ap.add_argument("--blobs", type=int, default=8)
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
g = ck.ClPlatforms.all().gpus()
m = MandelbrotRenderer(a.size, a.size, a.iters, devices=g[0])
m.render(1, pipeline=False)
flops = m.flops()
res = {"config": "mandelbrot_4k_1gpu", "size": a.size, "max_iter": a.iters, "flop": flops}
res["no_pipeline_ms"] = timeit(lambda: m.render(1, pipeline=False), a.reps)
res["event_pipeline_ms"] = timeit(lambda: m.render(2, pipeline=True, blobs=a.blobs), a.reps)
res["driver_pipeline_ms"] = timeit(lambda: m.render(3, pipeline=True, blobs=a.blobs,
                                                    pipeline_type=ck.PIPELINE_DRIVER), a.reps)
m.out.write = False
res["kernel_only_ms"] = timeit(lambda: m.render(4, pipeline=False), a.reps)
m.out.write = True
best = min(res["event_pipeline_ms"], res["driver_pipeline_ms"])
res["gflops_end_to_end"] = flops / (best * 1e-3) / 1e9
res["kernel_tflops"] = flops / (res["kernel_only_ms"] * 1e-3) / 1e12
res["kernel_pct_fp32_peak"] = 100 * res["kernel_tflops"] / FP32_PEAK_TFLOPS
res["d2h_bound_ms_at_55GBps"] = a.size * a.size * 4 / 55e9 * 1e3
emit(res)
