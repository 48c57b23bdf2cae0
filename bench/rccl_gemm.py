"""The RCCL (xGMI) data plane of one-process-per-GPU compute(), on the
8192³ bf16 GEMM: run under torchrun with one rank per GPU.

* ``split_reads``: every rank uploads 1/N of each full ``read`` array (A, B:
  128 MiB each) over its own PCIe link and one RCCL all-gather over xGMI
  completes every replica (instead of N whole uploads of each array);
  every rank downloads its C slice (host-resident GEMM).
* ``gather_writes``: the written C slices are all-gathered into every
  rank's device replica (the reference's "keep resident" iterative mode);
  rank 0 then checks sampled tiles from EVERY rank's range in its own
  replica against a float64 host product, which only passes if RCCL
  delivered the other ranks' slices.

Rank 0 prints one JSON line.  Host data are identical on every rank (same
seed), as split_reads requires."""
import argparse
import json
import time

import numpy as np

from common import sync

from cekirdekler_amd.ops.gemm import GEMM_LIBS, GemmBf16, from_bf16_bits, tile_coords
from cekirdekler_amd.ops.library import library
from cekirdekler_amd.parallel.distributed import DistributedCruncher, init_distributed

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=8192)
ap.add_argument("--steps", type=int, default=4)
ap.add_argument("--expect-world", type=int, default=0, help="fail unless the job has exactly this many ranks")
a = ap.parse_args()
ctx = init_distributed()
if a.expect_world and ctx.world != a.expect_world:
    raise SystemExit(f"rccl_gemm.py: expected {a.expect_world} ranks, the job has {ctx.world}")
import torch.distributed as dist  # noqa: E402

size = a.size
cr = DistributedCruncher("", ctx=ctx, prebuilt=library(*GEMM_LIBS), comm=True)
g = GemmBf16(size, size, size, cruncher=cr, tile="256x256pb")
cr.split_reads = True


def step():
    g.run(compute_id=5, resident=False)


step()
step()
if ctx.is_distributed:
    dist.barrier()
sync()
t0 = time.perf_counter()
for _ in range(a.steps):
    step()
sync()
ms = (time.perf_counter() - t0) * 1e3 / a.steps
rec = cr.last_record()
# host C slice of this rank vs float64
refs, rng = cr.references(5), cr.ranges(5)
unit = g.L * g.split_k
t_lo, nt = refs[ctx.rank] // unit, rng[ctx.rank] // unit
A = from_bf16_bits(g.A.array).reshape(size, size)
B = from_bf16_bits(g.B.array).reshape(size, size)
tile = g.BM * g.BN


def tile_err(c, t):
    r, col = tile_coords(np.array([t]), size, size, g.BM, g.BN, g.group_m)
    r, col = int(r[0]), int(col[0])
    ref = A[r * g.BM:(r + 1) * g.BM].astype(np.float64) @ B[col * g.BN:(col + 1) * g.BN].astype(np.float64).T
    got = g.tile_block(c[t * tile:(t + 1) * tile])
    return float(np.abs(got - ref).max() / np.abs(ref).max())


err_split = max(tile_err(g.C.array, t) for t in {t_lo, t_lo + nt - 1, t_lo + nt // 2}) if nt else 0.0
# gather_writes: device-resident C all-gathered into every replica
cr.split_reads = False
cr.gather_writes = True
g.run(compute_id=6, resident=False)  # A, B, C all moved; C slices then all-gathered
g.C.write = False
sync()
cr.download(g.C, 0)
refs6, rng6 = cr.references(6), cr.ranges(6)
picks = []
for r in range(ctx.world):
    lo, n = refs6[r] // unit, rng6[r] // unit
    if n:
        picks += [lo, lo + n - 1]
err_gather = max(tile_err(g.C.array, t) for t in picks)
rec6 = cr.last_record()
mine = (err_split, err_gather, ms, rec["h2d_bytes"], rec["d2h_bytes"], rec6["h2d_bytes"], rec6["d2h_bytes"])
errs = [mine]
if ctx.is_distributed:
    errs = [None] * ctx.world
    dist.all_gather_object(errs, mine)
if ctx.rank == 0:
    print(json.dumps({"config": "sgemm_host_resident_rccl", "ranks": ctx.world, "size": size,
                      "split_reads_ms": max(e[2] for e in errs),
                      "split_reads_tflops": 2 * size ** 3 / (max(e[2] for e in errs) * 1e-3) / 1e12,
                      "h2d_bytes_per_rank": [e[3] for e in errs],
                      "d2h_bytes_per_rank": [e[4] for e in errs],
                      "gather_call_h2d_bytes_per_rank": [e[5] for e in errs],
                      "gather_call_d2h_bytes_per_rank": [e[6] for e in errs],
                      "max_rel_err_split_reads": max(e[0] for e in errs),
                      "max_rel_err_gathered_replicas": max(e[1] for e in errs)}), flush=True)
cr.dispose()
if ctx.is_distributed:
    dist.barrier()
    dist.destroy_process_group()
