"""Multi-GPU tier: the xGMI paths on two or more PHYSICAL
MI355X.  Every test skips unless this process sees enough GPUs, so the tier
is inert on the one-GPU box and on the CPU tier; on an 8-GPU node it runs
before any benchmark does.

With ONE GPU the tier runs in rehearsal mode: the
"GPUs" are REHEARSAL_DEVICES logical devices on disjoint CU partitions of
GPU 0 (``ClDevices.cu_partitions``), every byte count, output and spread
assertion stands, and only the path assertions change — peer copies
between partitions of one GPU are ``local`` instead of ``xgmi``, the
topology has one ordinal.  The torchrun data-plane test then runs the same
worker logic over gloo with CPU devices (``TorchComm``) at world 2 and 4,
since RCCL refuses two ranks on one GPU.  With two or more GPUs nothing
changes.

Covered: the peer topology (hipDeviceCanAccessPeer + access enabled by
Cores), the single-process read fan-out over xGMI (reference: every device
uploads every ``read`` array, Worker.cs:833-860), the keep-resident gather
and ``share_slices`` between GPUs, a ClPipeline whose stages sit on distinct
GPUs (reference stage hand-over via host, ClPipeline.cs:1422-1574), a device
pool over every GPU, a range-partitioned bf16 GEMM over every GPU with its
output verified, and the RCCL data plane at world = N in a
torch.distributed.run child job.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import cekirdekler_amd as ck
from cekirdekler_amd.utils.multigpu import child_env, multi_gpu_skip_reason, torchrun_cmd, visible_gpus

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


PHYSICAL = visible_gpus() >= 2
REHEARSAL_DEVICES = 4
PATH = "xgmi" if PHYSICAL else "local"  # device-to-device path between the test's "GPUs"


def _need(n):
    why = multi_gpu_skip_reason(n)
    if why:
        pytest.skip(why)


@pytest.fixture
def gpus():
    g = ck.ClPlatforms.all().gpus()
    if PHYSICAL:
        return g
    if len(g) == 0:
        pytest.skip("no GPU visible")
    return g[0].cu_partitions(REHEARSAL_DEVICES)  # rehearsal: logical devices on disjoint CUs


def _all(gpus):
    devs = gpus[0]
    for i in range(1, len(gpus)):
        devs = devs + gpus[i]
    return devs


GATHER = """
__global__ void gather(const float* b, const int* nb, float* y) {
  long long i = get_global_id(0);
  int n = nb[0];
  y[i] = b[(i * 7919) % n] + 2.0f * b[n - 1 - (i % n)];
}
__global__ void hop(const float* x, float* y) {
  long long i = get_global_id(0);
  long long n = get_global_size(0);
  y[i] = x[(i * 7919) % n] * 0.5f + 1.0f;
}
"""


def test_peer_topology(gpus):
    cr = ck.ClNumberCruncher(_all(gpus), GATHER)
    topo = cr.peer_topology()
    n = len(gpus) if PHYSICAL else 1  # rehearsal: every logical device is GPU 0
    assert topo["ordinals"] == list(range(n))
    assert len(topo["matrix"]) == n and all(topo["matrix"][i][i] == 1 for i in range(n))
    if not PHYSICAL:
        assert topo["path"] == "none", topo
        cr.dispose()
        return
    assert topo["path"] in ("xgmi", "staged")
    # MI355X nodes: every GPU pair has a direct xGMI link
    assert topo["path"] == "xgmi", topo
    cr.dispose()


def test_read_fanout_across_gpus(gpus):
    n_dev = len(gpus)
    cr = ck.ClNumberCruncher(_all(gpus), GATHER)
    path = cr.peer_topology()["path"] if PHYSICAL else "local"
    nb = (3 << 20) // 4 * n_dev
    b = ck.ClArray(np.random.default_rng(0).standard_normal(nb).astype(np.float32))
    b.write = False
    nbv = ck.ClArray(np.array([nb], np.int32))
    nbv.write = False
    n_out = 256 * 64 * n_dev
    y = ck.ClArray(np.zeros(n_out, np.float32))
    y.read = False
    i = np.arange(n_out)
    for it in range(3):
        b.array[:] = b.array * np.float32(0.5) + np.float32(it)
        b.next_param(nbv, y).compute(cr, 1, "gather", n_out, 64)
        np.testing.assert_array_equal(y.array, b.array[(i * 7919) % nb] + np.float32(2) * b.array[nb - 1 - (i % nb)])
        rec = cr.last_record()
        if path in ("xgmi", "local"):
            assert rec["h2d_bytes"] == b.array.nbytes + n_dev * 4, rec
            assert rec["p2p_bytes"] == (n_dev - 1) * b.array.nbytes, rec
            assert rec["p2p_path"] == path and rec["staged_bytes"] == 0, rec
        else:  # explicit PCIe fallback: one whole upload per device
            assert rec["p2p_path"] == "pcie" and rec["h2d_bytes"] == n_dev * (b.array.nbytes + 4), rec
    cr.dispose()


def test_gather_flag_across_gpus(gpus):
    n_dev = len(gpus)
    cr = ck.ClNumberCruncher(_all(gpus), GATHER)
    cr.set_time_scale(n_dev - 1, 1.5)
    n = 1 << 20
    x0 = np.random.default_rng(1).standard_normal(n).astype(np.float32)
    a, b = ck.ClArray(x0.copy()), ck.ClArray(np.zeros(n, np.float32))
    for arr in (a, b):
        arr.write = False
        arr.gather_resident = True
    ref, src, dst = x0.copy(), a, b
    idx = (np.arange(n) * 7919) % n
    for it in range(8):
        src.read, dst.read = it == 0, False
        src.gather_resident, dst.gather_resident = False, True  # the written array
        src.next_param(dst).compute(cr, 2, "hop", n, 256)
        ref = ref[idx] * np.float32(0.5) + np.float32(1)
        rec = cr.last_record()
        if it:
            assert rec["h2d_bytes"] == 0 and rec["d2h_bytes"] == 0, rec
        assert rec["gather_bytes"] == (n_dev - 1) * n * 4, rec
        assert rec["p2p_path"] == PATH, rec  # MI355X: never host-staged
        src, dst = dst, src
    for d in range(n_dev):
        src.array[:] = 0
        cr.download(src, d)
        np.testing.assert_allclose(src.array, ref, rtol=1e-6, atol=1e-6)
    cr.dispose()


def test_share_slices_across_gpus(gpus):
    cr = ck.ClNumberCruncher(gpus[0] + gpus[1], GATHER)
    n = 1 << 18
    x0 = np.random.default_rng(2).standard_normal(n).astype(np.float32)
    a, b = ck.ClArray(x0.copy()), ck.ClArray(np.zeros(n, np.float32))
    a.write = b.write = False
    a.next_param(b).compute(cr, 3, "hop", n, 256)
    cr.cores.share_slices(3, b._spec(), 256)
    ref = x0[(np.arange(n) * 7919) % n] * np.float32(0.5) + np.float32(1)
    for d in range(2):
        b.array[:] = 0
        cr.download(b, d)
        np.testing.assert_allclose(b.array, ref, rtol=1e-6, atol=1e-6)
    cr.dispose()


def test_cl_pipeline_stages_on_distinct_gpus(gpus):
    from cekirdekler_amd.parallel.pipeline import ClPipelineStage

    n = 1 << 16
    k1 = "__global__ void f1(const float* x, float* y) { long long i = get_global_id(0); y[i] = x[i] * 2.0f + (float)i; }"
    k2 = "__global__ void f2(const float* y, float* z) { long long i = get_global_id(0); z[i] = y[i] + y[(i * 31) % 65536]; }"
    last = len(gpus) - 1
    s1, s2 = ClPipelineStage(), ClPipelineStage()
    s1.add_devices(gpus[0] + gpus[1] if len(gpus) > 2 else gpus[0])
    s1.add_kernels(k1, "f1", [n], [64])
    s1.add_input_buffers(np.zeros(n, np.float32))
    s1.add_output_buffers(np.zeros(n, np.float32))
    s2.add_devices(gpus[last])
    s2.add_kernels(k2, "f2", [n], [64])
    s2.add_input_buffers(np.zeros(n, np.float32))
    s2.add_output_buffers(np.zeros(n, np.float32))
    s1.prepend_to_stage(s2)
    pipe = s1.make_pipeline()
    i = np.arange(n)
    res, seen = np.zeros(n, np.float32), 0
    for p in range(10):
        if pipe.push_data([np.full(n, float(p), np.float32)], [res]):
            y = np.float32(seen) * 2 + i.astype(np.float32)
            np.testing.assert_array_equal(res, y + y[(i * 31) % n])
            seen += 1
    assert seen == 6
    st = pipe.transfer_stats()
    assert st["host"] == 0 and st["p2p"] > 0, st
    pipe.dispose()


def test_device_pool_over_every_gpu(gpus):
    from cekirdekler_amd.parallel.pool import ClDevicePool, ClDevicePoolType, ClTaskPool

    src = "__global__ void fill(float* x, float* v) { x[get_global_id(0)] = v[0] * 2.0f; }"
    pool = ClDevicePool(ClDevicePoolType.DEVICE_COMPUTE_AT_WILL, src, False, 3)
    pool.add_device(_all(gpus))
    tp = ClTaskPool()
    arrays = []
    for t in range(16 * len(gpus)):
        x = ck.ClArray(np.zeros(4096, np.float32))
        v = ck.ClArray(np.array([t], np.float32))
        v.write = False
        tp.feed(x.next_param(v).task(1, "fill", 4096, 64))
        arrays.append(x)
    pool.enqueue_task_pool(tp)
    pool.finish()
    for t, x in enumerate(arrays):
        np.testing.assert_array_equal(x.array, 2.0 * t)
    counts = pool.device_task_counts()
    assert sum(counts) == 16 * len(gpus) and sum(1 for c in counts if c) >= 2, counts
    pool.dispose()


def test_gemm_over_every_gpu_verified(gpus):
    from cekirdekler_amd.ops.gemm import GemmBf16

    g = GemmBf16(2048, 2048, 2048, devices=_all(gpus), tile="256x256pb")
    for _ in range(3):
        g.run(resident=True)
    assert g.verify() < 1e-4
    assert all(r > 0 for r in g.cr.ranges(1)), g.cr.ranges(1)
    g.run(resident=False)
    c, ref = g.result(download=False), g.reference()
    assert np.abs(c - ref).max() < 1e-4 * np.abs(ref).max()
    g.cr.dispose()


@pytest.mark.parametrize("nproc", [2, 0])
def test_rccl_data_plane_torchrun(nproc):
    """torch.distributed.run child job, one rank per GPU (nproc 0: all of
    them): broadcast_reads, split_reads, gather_writes with uneven splits,
    and the keep-resident gather flag; every rank checks its replicas."""
    if not PHYSICAL:
        if visible_gpus() == 0:
            pytest.skip("no GPU visible (the CPU tier runs this rehearsal: test_multi_gating.py)")
        # rehearsal: the same worker checks over gloo on CPU devices
        # (TorchComm), ranks 2 and 4 (RCCL refuses two ranks on one GPU)
        n = nproc or REHEARSAL_DEVICES
        cmd = torchrun_cmd(os.path.join(HERE, "rccl_worker.py"), n, ["--torchcomm"])
        env = child_env()
        env["CEK_CPU_THREADS"] = "2"
        r = subprocess.run(cmd, cwd=HERE, env=env, capture_output=True, text=True, timeout=240)
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        assert r.returncode == 0 and lines, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
        out = json.loads(lines[-1])
        assert out["ok"] and out["ranks"] == n, json.dumps(out)[:3000]
        assert out["per_rank"][0]["uneven"], out["per_rank"][0]
        assert all(o["backend"] == "gloo" for o in out["per_rank"])
        return
    n = nproc or visible_gpus()
    _need(max(2, n))
    cmd = torchrun_cmd(os.path.join(HERE, "rccl_worker.py"), n)
    r = subprocess.run(cmd, cwd=HERE, env=child_env(), capture_output=True, text=True, timeout=240)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and lines, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    out = json.loads(lines[-1])
    assert out["ok"] and out["ranks"] == n, json.dumps(out)[:3000]
    assert out["per_rank"][0]["uneven"], out["per_rank"][0]
    assert sorted(o["gpu_ordinal"] for o in out["per_rank"]) == list(range(n))


def test_xgmi_link_bandwidth_floor(gpus):
    """measured, not assumed.  Each timed pair moves 256 MiB
    GPU→GPU with both engines, byte-exact, and the faster engine clears a
    loose floor of 50 GB/s (one xGMI link ≈ 153 GB/s peak); every ordered
    pair at once must beat one pair alone (the links are point to point)."""
    from cekirdekler_amd.utils.multigpu import peer_bandwidth_report

    if not PHYSICAL:  # rehearsal: the same measurement inside GPU 0 (no link to be bound by)
        rep = peer_bandwidth_report([0, 0], reps=3)
        assert rep["all_verified"], rep
        assert rep["min_pair_gbps"] >= 50.0, rep
        return
    rep = peer_bandwidth_report(list(range(len(gpus))), reps=3)
    assert rep["all_verified"], rep
    assert rep["min_pair_gbps"] >= 50.0, rep
    best_all = max(v["aggregate_gbps"] for v in rep["all_pairs"].values())
    assert best_all > rep["min_pair_gbps"], rep
