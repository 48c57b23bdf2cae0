"""Few dispatches of the VALU-bound kernels (Mandelbrot $MANDEL_KERNELS, N-body b2/b4)
for counter collection under rocprofv3 --pmc."""
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.models.mandelbrot import MandelbrotRenderer  # noqa: E402
from cekirdekler_amd.models.nbody import NBodySimulation  # noqa: E402

g0 = ck.ClPlatforms.all().gpus()[0]
import os
for kern in os.environ.get("MANDEL_KERNELS", "blk8k,blk8t").split(","):
    m = MandelbrotRenderer(4096, 4096, 256, devices=g0, kernel=kern)
    m.out.write = False
    for _ in range(3):
        m.render(1, pipeline=False)
    torch.cuda.synchronize()
    m.cr.dispose()
for b in ((2, 4) if os.environ.get("NBODY", "1") == "1" else ()):
    sim = NBodySimulation(262144, devices=g0, bodies_per_item=b)
    for _ in range(2):
        sim.forces()
    torch.cuda.synchronize()
