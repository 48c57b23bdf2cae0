"""The load balancer gets each GPU's device time (hipEvent spans around its
work) instead of host wall clock:
in enqueue mode, devices of one process are credited with their own spans,
so heterogeneity re-balances from enqueue-mode runs."""
import numpy as np
import pytest

import cekirdekler_amd as ck

pytestmark = pytest.mark.gpu

SKEW = """
__global__ void skew(float* x, const int* n) {
  long long i = get_global_id(0);
  int reps = (i >= n[0] / 2) ? 6000 : 600;   // the upper half costs 10x
  float v = x[i];
  for (int k = 0; k < reps; ++k) v = v * 0.9999f + 0.25f;
  x[i] = v;
}
"""


@pytest.mark.parametrize("mode", ["sync", "enqueue"])
def test_uneven_work_rebalances_by_device_time(mode):
    g0 = ck.ClPlatforms.all().gpus()[0]
    cr = ck.ClNumberCruncher(g0 + g0, SKEW)
    cr.cores.serial = True  # logical devices of one GPU: sync computes timed in isolation
    n = 1 << 20
    x = ck.ClArray(np.zeros(n, np.float32))
    x.read = x.write = False
    nv = ck.ClArray(np.array([n], np.int32))
    nv.write = False
    x.next_param(nv).compute(cr, 1, "skew", n, 256)  # equal split
    assert cr.ranges(1) == [n // 2, n // 2]
    for _ in range(6):
        if mode == "enqueue":
            cr.enqueue_mode = True  # the split is frozen while enqueueing
            for _ in range(3):
                x.next_param(nv).compute(cr, 1, "skew", n, 256)
            cr.enqueue_mode = False  # each device credited with its own spans here
            b = cr.benchmarks(1)
            # Logical devices of one GPU share its hardware queues, so their
            # spans overlap; on separate GPUs each is its own device time.
            assert all(v > 0 for v in b), b
        x.next_param(nv).compute(cr, 1, "skew", n, 256)  # re-balances from those timings
    r = cr.ranges(1)
    assert r[0] > 1.3 * r[1], r  # device 0 (cheap half) takes more work items
    cr.dispose()
