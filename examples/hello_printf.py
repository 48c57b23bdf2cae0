"""The reference README's first example: a kernel that prints from every work
item (global 1000, local 100), on every GPU or the CPU device."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402

SRC = """
__kernel void hello(__global char* arr)
{
    printf("hello world\\n");
}"""
plats = ck.ClPlatforms.all()
devices = plats.gpus() if len(plats.gpus()) else plats.cpus(True)
cr = ck.ClNumberCruncher(devices, SRC)
arr = ck.ClArray(np.zeros(1000, np.uint8))
arr.read = arr.write = False
arr.compute(cr, 1, "hello", 1000, 100)
cr.dispose()
