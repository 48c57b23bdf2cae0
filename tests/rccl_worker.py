"""One rank of the multi-rank data-plane check (started by torch.distributed.run
from tests/test_gpu_multi.py, one rank per GPU; or on CPU devices with gloo
from tests/test_multi_gating.py as a control-plane rehearsal).

GPU mode exercises DistributedCruncher's RCCL data plane at world > 1:

* ``broadcast_reads``: only rank 0's host copy holds the data (the others
  hold zeros); rank 0 uploads, RCCL broadcasts over xGMI;
* ``split_reads``: identical host copies; each rank uploads 1/N, RCCL
  all-gathers;
* ``gather_writes``: written slices all-gathered into every rank's device
  replica — with uneven splits (a time scale per rank) this runs the grouped
  broadcast branch of ``Comm::allgatherv`` (csrc/dist.cpp);
* the per-array ``gather`` flag (keep-resident): iterative ping-pong with no
  host transfer after the first call.

Every rank downloads its replicas and compares ALL elements with numpy (so a
slice RCCL failed to deliver shows up on the rank that misses it).  Rank 0
prints one JSON line with every rank's verdict.
"""
import argparse
import json
import sys

import numpy as np

SRC = """
__global__ void k(const float* a, float* y) {
  long long i = get_global_id(0);
  long long n = get_global_size(0);
  y[i] = a[(i * 7919) % n] * 3.0f + 1.0f;
}
"""


def ref_k(a):
    n = len(a)
    return a[(np.arange(n) * 7919) % n] * np.float32(3.0) + np.float32(1.0)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpu", action="store_true", help="control-plane rehearsal on CPU devices (gloo)")
    ap.add_argument("--torchcomm", action="store_true",
                    help="data-plane rehearsal: every GPU-mode check on CPU devices, collectives over gloo "
                         "(TorchComm; the host array is each rank's replica)")
    ap.add_argument("--elems", type=int, default=256 * 1024)
    a = ap.parse_args()
    import cekirdekler_amd as ck
    from cekirdekler_amd.parallel.distributed import DistributedCruncher, init_distributed

    tc = a.torchcomm
    ctx = init_distributed("gloo" if (a.cpu or tc) else None)
    import torch.distributed as dist

    rank, world, n = ctx.rank, ctx.world, a.elems
    checks = {}
    info = {"rank": rank, "backend": ctx.backend}
    try:
        if a.cpu:
            cr = DistributedCruncher(SRC, ctx=ctx, devices=ck.ClPlatforms.all().cpus(True))
        elif tc:
            cr = DistributedCruncher(SRC, ctx=ctx, devices=ck.ClPlatforms.all().cpus(True), comm=True)
            info["comm"] = type(cr._comm).__name__
        else:
            cr = DistributedCruncher(SRC, ctx=ctx, comm=True)
            info["gpu_ordinal"] = cr.devices.device(0).info.ordinal
        cr.set_time_scale(0, 1.0 + 0.6 * rank)  # uneven splits after the first call
        rng = np.random.default_rng(7)
        data = rng.standard_normal(n).astype(np.float32)
        splits = []
        # 1) broadcast_reads + gather_writes, uneven splits
        x = ck.ClArray(data.copy() if rank == 0 or a.cpu else np.zeros(n, np.float32))
        replica = (lambda arr: None) if tc else (lambda arr: (arr.array.fill(0), cr.download(arr, 0)))
        x.write = False
        y = ck.ClArray(np.zeros(n, np.float32))
        y.read = False
        if not a.cpu:
            cr.broadcast_reads = True
            cr.gather_writes = True
        for _ in range(5):
            x.next_param(y).compute(cr, 1, "k", n, 256)
            splits.append(list(cr.ranges(1)))
        info["ranges"] = splits[-1]
        info["uneven"] = len(set(splits[-1])) > 1
        want = ref_k(data)
        lo, hi = cr.references(1)[rank], cr.references(1)[rank] + cr.ranges(1)[rank]
        if a.cpu:
            checks["own_slice"] = bool(np.array_equal(y.array[lo:hi], want[lo:hi]))
        else:
            checks["host_replica_all"] = bool(np.array_equal(y.array, want))
            replica(y)
            checks["device_replica_all"] = bool(np.array_equal(y.array, want))
            rec = cr.last_record()
            info["broadcast_h2d_bytes"] = rec["h2d_bytes"]
            cr.broadcast_reads = False
            cr.gather_writes = False
            # 2) split_reads: identical host copies, 1/N uploaded per rank
            x2 = ck.ClArray(data.copy())
            x2.write = False
            cr.split_reads = True
            y.array[:] = 0
            x2.next_param(y).compute(cr, 2, "k", n, 256)
            x2.next_param(y).compute(cr, 2, "k", n, 256)
            lo, hi = cr.references(2)[rank], cr.references(2)[rank] + cr.ranges(2)[rank]
            checks["split_reads_slice"] = bool(np.array_equal(y.array[lo:hi], want[lo:hi]))
            info["split_h2d_bytes"] = cr.last_record()["h2d_bytes"]
            cr.split_reads = False
            # 3) keep-resident gather flag: ping-pong, no host traffic after call 1
            p = ck.ClArray(data.copy())
            q = ck.ClArray(np.zeros(n, np.float32))
            for arr in (p, q):
                arr.write = False
                arr.gather_resident = True
            src, dst, ref = p, q, data.copy()
            moved = []
            for it in range(6):
                src.read = it == 0
                dst.read = False
                src.gather_resident, dst.gather_resident = False, True
                src.next_param(dst).compute(cr, 3, "k", n, 256)
                ref = ref_k(ref)
                r = cr.last_record()
                moved.append(r["h2d_bytes"] + r["d2h_bytes"])
                src, dst = dst, src
            replica(src)
            # float chains: compare with a tolerance (kernel fma vs numpy)
            checks["gather_flag_replica"] = bool(np.allclose(src.array, ref, rtol=1e-4, atol=1e-4))
            checks["gather_flag_no_host_traffic"] = all(m == 0 for m in moved[1:])

        cr.dispose()
    except Exception as e:  # report, never hang the other ranks
        checks["exception"] = False
        info["error"] = repr(e)[:400]
    info["checks"] = checks
    info["ok"] = bool(checks) and all(checks.values())
    out = [None] * world
    dist.all_gather_object(out, info)
    if rank == 0:
        same = all(o.get("ranges") == out[0].get("ranges") for o in out)
        print(json.dumps({"ranks": world, "ok": all(o["ok"] for o in out) and same,
                          "splits_identical": same, "per_rank": out}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0 if all(o["ok"] for o in out) else 1


if __name__ == "__main__":
    sys.exit(main())
