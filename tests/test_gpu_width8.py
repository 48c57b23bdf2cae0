"""Width-8 rehearsal on one GPU: every multi-device path at the node's real
width (8 MI355X), as 8 logical devices of GPU 0 (the reference allows the
same device several times: ClPipeline.cs:4337, :1728; ClObjectApi.cs:813).

The 8-wide loops of the read fan-out, the keep-resident gather, the
per-device event vectors, the stage pipeline with 8-device stages, a device
pool with 8 consumers and a range-partitioned GEMM over 8 devices run here
exactly as they would over xGMI (peer copies become D2D copies of one GPU).
"""
import numpy as np
import pytest

import cekirdekler_amd as ck

pytestmark = pytest.mark.gpu

W = 8

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


def _w(k=W):
    g0 = ck.ClPlatforms.all().gpus()[0]
    devs = g0
    for _ in range(k - 1):
        devs = devs + g0
    return devs


def test_read_fanout_8():
    cr = ck.ClNumberCruncher(_w(), GATHER)
    nb = (3 << 20) // 4 * W
    b = ck.ClArray(np.random.default_rng(0).standard_normal(nb).astype(np.float32))
    b.write = False
    nbv = ck.ClArray(np.array([nb], np.int32))
    nbv.write = False
    n_out = 256 * 64 * W
    y = ck.ClArray(np.zeros(n_out, np.float32))
    y.read = False
    i = np.arange(n_out)
    for it in range(3):
        b.array[:] = b.array * np.float32(0.5) + np.float32(it)
        b.next_param(nbv, y).compute(cr, 1, "gather", n_out, 64)
        want = b.array[(i * 7919) % nb] + np.float32(2.0) * b.array[nb - 1 - (i % nb)]
        np.testing.assert_array_equal(y.array, want)
        rec = cr.last_record()
        assert rec["h2d_bytes"] == b.array.nbytes + W * 4, rec
        assert rec["p2p_bytes"] == (W - 1) * b.array.nbytes, rec
        assert len(rec["ranges"]) == W and all(r > 0 for r in rec["ranges"])
    cr.dispose()


@pytest.mark.parametrize("enqueue", [False, True])
def test_gather_ping_pong_8(enqueue):
    cr = ck.ClNumberCruncher(_w(), GATHER)
    cr.set_time_scale(W - 1, 1.7)
    n = 1 << 17
    x0 = np.random.default_rng(2).standard_normal(n).astype(np.float32)
    a, b = ck.ClArray(x0.copy()), ck.ClArray(np.zeros(n, np.float32))
    a.write = b.write = False
    ref, src, dst = x0.copy(), a, b
    idx = (np.arange(n) * 7919) % n
    src.read, dst.read = True, False
    src.gather_resident, dst.gather_resident = False, True
    src.next_param(dst).compute(cr, 2, "hop", n, 64)  # the balancer moves off the equal split
    ref = ref[idx] * np.float32(0.5) + np.float32(1)
    src, dst = dst, src
    for it in range(4):  # sync calls: re-balanced splits
        src.read = dst.read = False
        src.gather_resident, dst.gather_resident = False, True
        src.next_param(dst).compute(cr, 2, "hop", n, 64)
        ref = ref[idx] * np.float32(0.5) + np.float32(1)
        assert cr.last_record()["gather_bytes"] == (W - 1) * n * 4
        src, dst = dst, src
    if enqueue:
        cr.enqueue_mode = True
    for it in range(6):
        src.gather_resident, dst.gather_resident = False, True
        src.next_param(dst).compute(cr, 2, "hop", n, 64)
        ref = ref[idx] * np.float32(0.5) + np.float32(1)
        src, dst = dst, src
    if enqueue:
        cr.enqueue_mode = False
    assert len(set(cr.ranges(2))) > 1
    for d in range(W):
        src.array[:] = 0
        cr.download(src, d)
        np.testing.assert_allclose(src.array, ref, rtol=1e-6, atol=1e-6)
    cr.dispose()


def test_cl_pipeline_8_device_stages():
    """Two stages of 8 logical devices each (uneven split in stage 1): every
    transition is a device→device copy, nothing staged through the host."""
    from cekirdekler_amd.parallel.pipeline import ClPipelineStage

    n = 1 << 16
    k1 = "__global__ void f1(const float* x, float* y) { long long i = get_global_id(0); y[i] = x[i] * 3.0f + (float)i; }"
    k2 = "__global__ void f2(const float* y, float* z) { long long i = get_global_id(0); z[i] = y[i] + y[(i * 31) % 65536]; }"
    s1, s2 = ClPipelineStage(), ClPipelineStage()
    s1.add_devices(_w())
    s1.add_kernels(k1, "f1", [n], [64])
    s1.add_input_buffers(np.zeros(n, np.float32))
    s1.add_output_buffers(np.zeros(n, np.float32))
    s2.add_devices(_w())
    s2.add_kernels(k2, "f2", [n], [64])
    s2.add_input_buffers(np.zeros(n, np.float32))
    s2.add_output_buffers(np.zeros(n, np.float32))
    s1.prepend_to_stage(s2)
    pipe = s1.make_pipeline()
    s1.cruncher.set_time_scale(W - 1, 2.5)
    i = np.arange(n)

    def expect(p):
        y = np.float32(3.0) * np.float32(p) + i.astype(np.float32)
        return y + y[(i * 31) % n]

    res = np.zeros(n, np.float32)
    seen = 0
    pushes = 10
    for p in range(pushes):
        if pipe.push_data([np.full(n, float(p), np.float32)], [res]):
            np.testing.assert_array_equal(res, expect(seen))
            seen += 1
    assert seen == pushes - 4
    st = pipe.transfer_stats()
    assert st["host"] == 0 and st["p2p"] > 0
    assert len(set(s1.cruncher.ranges(1))) > 1
    pipe.dispose()


@pytest.mark.parametrize("policy", ["DEVICE_COMPUTE_AT_WILL", "DEVICE_ROUND_ROBIN"])
def test_device_pool_8_consumers(policy):
    from cekirdekler_amd.parallel.pool import ClDevicePool, ClDevicePoolType, ClTaskPool

    src = "__global__ void fill(float* x, float* v) { x[get_global_id(0)] = v[0] + (float)get_global_id(0); }"
    pool = ClDevicePool(getattr(ClDevicePoolType, policy), src, True, 4)
    pool.add_device(_w())
    tp = ClTaskPool()
    xs = []
    for k in range(256):
        x = ck.ClArray(np.zeros(1024, np.float32))
        v = ck.ClArray(np.array([float(k)], np.float32))
        v.write = False
        tp.feed(x.next_param(v).task(1, "fill", 1024, 256))
        xs.append(x)
    pool.enqueue_task_pool(tp)
    pool.finish()
    for k, x in enumerate(xs):
        np.testing.assert_array_equal(x.array, float(k) + np.arange(1024, dtype=np.float32))
    counts = pool.device_task_counts()
    assert sum(counts) == 256 and len(counts) == W
    if policy == "DEVICE_ROUND_ROBIN":
        assert counts == [32] * W
    else:
        assert sum(c > 0 for c in counts) >= 2
    pool.dispose()


def test_gemm_over_8_logical_devices_verified():
    """A range-partitioned bf16 GEMM split 8 ways (wave-quantized balancing
    off: one-tile units so every device gets a share), one device slower,
    checked against a float64 product on every device's tiles."""
    from cekirdekler_amd.ops.gemm import GEMM_LIBS, GemmBf16
    from cekirdekler_amd.ops.library import library

    cr = ck.ClNumberCruncher(_w(), "", prebuilt=library(*GEMM_LIBS))
    cr.set_time_scale(3, 1.8)
    g = GemmBf16(2048, 2048, 1024, cruncher=cr, tile="256x256pb", wave_granularity=False)
    for _ in range(4):
        g.run(compute_id=1, resident=True)
    r = cr.ranges(1)
    assert len(r) == W and all(x > 0 for x in r) and sum(r) == g.global_range
    assert g.verify(compute_id=1, tiles_per_device=4) < 1e-4
    cr.dispose()
