"""Host cost of one hipModuleLaunchKernel by argument mode, before and after
the process has loaded the library code objects (tools/pool_env_probe.py:
one pool consumer's issue cost triples once they are loaded).

    python tools/launch_mode_probe.py > gpurun_out/launch_mode.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd._native import cek  # noqa: E402
from cekirdekler_amd.ops.library import code_object, library  # noqa: E402


def us(mode):
    r = cek.launch_rate_probe(0, code_object("stream"), "cek_copy_u8", 1, 4000, mode)
    return round(1e3 * r["host_ms"] / 4000, 3)


out = {"before": {"kernel_params": us(0), "packed": us(1)}}
cr = ck.ClNumberCruncher(ck.ClPlatforms.all().gpus()[0], "", prebuilt=library("sgemm_bf16", "reduce", "nbody",
                                                                              "mandelbrot", "stream"))
out["after_libs"] = {"kernel_params": us(0), "packed": us(1)}
cr.dispose()
out["after_dispose"] = {"kernel_params": us(0), "packed": us(1)}
print(json.dumps(out), flush=True)
