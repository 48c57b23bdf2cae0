"""Few fp32 GEMM dispatches for counter collection under rocprofv3 --pmc.
usage: python tools/gemm_f32_pmc.py [tile,...]   (default 256x256)"""
import sys
sys.path.insert(0, '.')
import torch
import cekirdekler_amd as ck
from cekirdekler_amd.ops.gemm import GemmF32
g0 = ck.ClPlatforms.all().gpus()[0]
tiles = sys.argv[1].split(",") if len(sys.argv) > 1 else ["256x256"]
for tile in tiles:
    g = GemmF32(8192, 8192, 8192, devices=g0, tile=tile, group_m=4)
    for _ in range(3):
        g.run(resident=True)
    torch.cuda.synchronize()
    g.cr.dispose()
if "torch" in sys.argv[1:]:
    a = torch.randn(8192, 8192, device="cuda")
    b = torch.randn(8192, 8192, device="cuda")
    for _ in range(3):
        torch.matmul(a, b.t())
    torch.cuda.synchronize()
