"""Few GEMM dispatches for counter collection under rocprofv3 --pmc.
usage: python tools/gemm_pmc.py [tile[@rows],...]   (default 256x256pp; rows = M, default 8192)"""
import sys
sys.path.insert(0, '.')
import torch
import cekirdekler_amd as ck
from cekirdekler_amd.ops.gemm import GemmBf16
g0 = ck.ClPlatforms.all().gpus()[0]
tiles = sys.argv[1].split(",") if len(sys.argv) > 1 else ["256x256pp"]
for spec in tiles:
    tile, _, rows = spec.partition("@")
    g = GemmBf16(int(rows or 8192), 8192, 8192, devices=g0, tile=tile, group_m=4)
    for _ in range(3):
        g.run(resident=True)
    torch.cuda.synchronize()
    g.cr.dispose()
