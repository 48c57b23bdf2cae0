"""Few GEMM dispatches for counter collection under rocprofv3."""
import sys
sys.path.insert(0, '.')
import torch
import cekirdekler_amd as ck
from cekirdekler_amd.ops.gemm import GemmBf16
g0 = ck.ClPlatforms.all().gpus()[0]
for tile, gm in [("256x256", 1), ("256x256", 4), ("256x256pp", 4)]:
    g = GemmBf16(8192, 8192, 8192, devices=g0, tile=tile, group_m=gm)
    for _ in range(3):
        g.run(resident=True)
    torch.cuda.synchronize()
    g.cr.dispose()
