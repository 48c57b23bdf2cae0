"""One-process-per-device range partitioning across ranks (gloo, world 2):
both ranks derive identical splits from exchanged timings (shared-memory
control plane and the torch.distributed fallback)."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.multiprocessing as mp  # noqa: E402

SRC = """
__global__ void k(float* x) { long long i = get_global_id(0); x[i] = x[i] * 2.0f + (float)i; }
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, exch, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), CEK_CPU_THREADS="2")
    import cekirdekler_amd as ck
    from cekirdekler_amd.parallel.distributed import DistributedCruncher, init_distributed

    ctx = init_distributed("gloo")
    cr = DistributedCruncher(SRC, ctx=ctx, devices=ck.ClPlatforms.all().cpus(True), exchanger=exch)
    if rank == 1:
        cr.set_time_scale(0, 3.0)  # rank 1's device looks 3x slower
    n = 64 * 512
    x = ck.ClArray(np.ones(n, np.float32))
    splits = []
    import warnings
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        for it in range(12):
            x.array[:] = 1.0  # read whole + written by slices: fine only because it is reset
            x.compute(cr, 1, "k", n, 64)
            splits.append(cr.ranges(1))
    warned = sum("read whole and written by slices" in str(w.message) for w in caught)
    # enqueue mode (no per-call exchange) is entered and left by every rank
    # together; the timings gathered on leaving keep the splits identical
    cr.enqueue_mode = True
    for _ in range(3):
        x.compute(cr, 1, "k", n, 64)
    cr.enqueue_mode = False
    for _ in range(2):
        x.array[:] = 1.0
        x.compute(cr, 1, "k", n, 64)
        splits.append(cr.ranges(1))
    refs = cr.references(1)
    lo, hi = refs[rank], refs[rank] + splits[-1][rank]
    ok = bool(np.all(x.array[lo:hi] == 2.0 + np.arange(lo, hi, dtype=np.float32)))
    q.put((rank, splits, ok and warned == 1))
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("exch,world", [("shm", 2), ("torch", 2), ("shm", 4)])
def test_two_rank_balancing(exch, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, exch, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, splits, ok = q.get(timeout=240)
        res[r] = (splits, ok)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for r in range(1, world):
        assert res[r][0] == res[0][0]      # identical splits on every rank, every call
    assert all(res[r][1] for r in range(world))  # each rank computed its own slice correctly
    last = res[0][0][-1]
    assert sum(last) == 64 * 512 and last[0] > last[1]  # faster rank 0 got more work
