"""One process per device on the GPU: two ranks (gloo control plane, both on
GPU 0 of the test box) run DistributedCruncher computes — library GEMM and a
JIT kernel — with identical splits on both ranks and correct slices."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.multiprocessing as mp  # noqa: E402

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        import cekirdekler_amd as ck
        from cekirdekler_amd.ops.gemm import GEMM_LIBS, GemmBf16
        from cekirdekler_amd.ops.library import library
        from cekirdekler_amd.parallel.distributed import DistributedCruncher, init_distributed

        ctx = init_distributed("gloo")
        gpu = ck.ClPlatforms.all().gpus()[0]
        cr = DistributedCruncher("", ctx=ctx, devices=gpu, prebuilt=library(*GEMM_LIBS))
        g = GemmBf16(1024, 512, 512, cruncher=cr, tile="256x256pb")
        splits = []
        for _ in range(4):
            g.run(resident=False)
            splits.append(cr.ranges(1))
        c = g.result(download=False)
        ref = g.reference()
        refs, rng = cr.references(1), cr.ranges(1)
        e = g.C.elements_per_work_item
        # rows of this rank's tiles: compare the tile-major slice it wrote
        from cekirdekler_amd.ops.gemm import untile
        mine = np.zeros_like(g.C.array)
        lo, hi = refs[rank] * e, (refs[rank] + rng[rank]) * e
        mine[lo:hi] = 1
        mask = untile(mine, g.M, g.N, g.BM, g.BN, g.group_m, g.geom) > 0
        ok = bool(np.abs(c[mask] - ref[mask]).max() < 1e-4 * np.abs(ref).max()) if mask.any() else True
        src = "__global__ void k(float* x) { long long i = get_global_id(0); x[i] = x[i] * 2.0f + 1.0f; }"
        cj = DistributedCruncher(src, ctx=ctx, devices=gpu)
        n = 256 * 64
        x = ck.ClArray(np.ones(n, np.float32))
        for _ in range(3):
            x.array[:] = 1.0
            x.compute(cj, 3, "k", n, 256)
        r3 = cj.references(3)
        lo, hi = r3[rank], r3[rank] + cj.ranges(3)[rank]
        ok2 = bool(np.all(x.array[lo:hi] == 3.0))
        q.put((rank, splits, ok and ok2, ""))
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()
    except Exception as ex:  # report instead of hanging the parent
        q.put((rank, None, False, repr(ex)))


def test_two_ranks_share_gpu0():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, splits, ok, err = q.get(timeout=300)
        res[r] = (splits, ok, err)
    for p in procs:
        p.join(120)
    assert res[0][1] and res[1][1], (res[0][2], res[1][2])
    assert res[0][0] == res[1][0]
    assert all(sum(s) == 2 * 4 * 512 for s in res[0][0])


def test_rccl_data_plane_one_rank():
    """The RCCL data plane of DistributedCruncher (rank-0 upload + broadcast of
    ``read`` arrays, in-place all-gather-v of written slices into the device
    replica) on a one-rank communicator, plus the raw Comm collectives on
    torch device memory.  Multi-rank RCCL needs one GPU per rank."""
    import cekirdekler_amd as ck
    from cekirdekler_amd._native import cek
    from cekirdekler_amd.parallel.distributed import DistContext, DistributedCruncher

    gpu = ck.ClPlatforms.all().gpus()[0]
    src = """__global__ void k(const float* a, float* y) {
        long long i = get_global_id(0); y[i] = a[i] * 3.0f + 1.0f; }"""
    cr = DistributedCruncher(src, ctx=DistContext(), devices=gpu, comm=True)
    cr.broadcast_reads = True
    cr.gather_writes = True
    n = 256 * 64
    a = ck.ClArray(np.arange(n, dtype=np.float32))
    a.write = False
    y = ck.ClArray(np.zeros(n, np.float32))
    y.read = False
    for _ in range(3):
        a.next_param(y).compute(cr, 1, "k", n, 256)
    np.testing.assert_allclose(y.array, np.arange(n, dtype=np.float32) * 3 + 1)
    cr.download(y, 0)  # the gathered device replica holds every slice
    np.testing.assert_allclose(y.array, np.arange(n, dtype=np.float32) * 3 + 1)
    cr.dispose()

    # split upload + all-gather of full reads (one rank: the whole array is
    # its chunk; the all-gather is the identity)
    cr = DistributedCruncher(src, ctx=DistContext(), devices=gpu, comm=True)
    cr.split_reads = True
    a = ck.ClArray(np.arange(n + 3 * 64, dtype=np.float32))  # odd size: uneven chunks at N ranks
    a.write = False
    y = ck.ClArray(np.zeros(n, np.float32))
    y.read = False
    for _ in range(2):
        a.next_param(y).compute(cr, 2, "k", n, 256)
    np.testing.assert_allclose(y.array, np.arange(n, dtype=np.float32) * 3 + 1)
    assert cr.last_record()["h2d_bytes"] == a.array.nbytes
    cr.dispose()

    comm = cek.RcclComm(cek.RcclComm.unique_id(), 0, 1, gpu.device(0).info.ordinal)
    t = torch.arange(1024, dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    comm.allreduce_sum_f32(t.data_ptr(), t.numel(), s)
    comm.broadcast(t.data_ptr(), t.numel() * 4, 0, s)
    torch.cuda.synchronize()
    assert torch.equal(t.cpu(), torch.arange(1024, dtype=torch.float32))
