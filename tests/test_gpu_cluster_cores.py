"""GPU tier for the reference's other entry points: the "usage type 2"
``Cores`` API on GPU / CPU+GPU with each pipeline kind, and the cluster
layer (loopback TCP servers whose nodes compute on the MI355X)."""
import numpy as np
import pytest

import cekirdekler_amd as ck
from cekirdekler_amd.parallel.cluster import ClCruncherServer, ClusterAccelerator, find_servers

pytestmark = pytest.mark.gpu

SRC = """
__global__ void saxpy(const float* a, const float* x, float* y) {
  long long i = get_global_id(0);
  y[i] = a[0] * x[i] + y[i];
}
"""


@pytest.mark.parametrize("types", ["gpu", "cpu gpu"])
@pytest.mark.parametrize("pipeline,ptype", [(False, True), (True, ck.PIPELINE_EVENT), (True, ck.PIPELINE_DRIVER)])
def test_cores_usage_type_2_gpu(types, pipeline, ptype):
    cores = ck.Cores(types, SRC, local_range=64)
    n = 64 * 16 * 64
    a = np.array([2.0], np.float32)
    x = np.arange(n, dtype=np.float32)
    for _ in range(3):
        y = np.ones(n, np.float32)
        cores.compute("saxpy", 1, "", [a, x, y], [" read ", " partial read ", " partial read write "], [1, 1, 1],
                      n, 1, 0, pipeline, 4, ptype)
        np.testing.assert_array_equal(y, 2 * x + 1)
    assert "Compute-ID: 1" in cores.performance_report(1)
    cores.dispose()


def test_cluster_nodes_compute_on_gpu():
    servers = [ClCruncherServer(0, "127.0.0.1").start() for _ in range(2)]
    try:
        nodes = find_servers(["127.0.0.1"], [s.port for s in servers])
        assert len(nodes) == 2
        acc = ClusterAccelerator()
        acc.setup_nodes(nodes, "gpu", SRC, ["saxpy"], 64, mainframe_types="gpu")
        n = 64 * 1000 + 64 * 3
        a = np.array([2.0], np.float32)
        x = np.arange(n, dtype=np.float32)
        for _ in range(4):
            y = np.ones(n, np.float32)
            acc.compute("saxpy", 1, "", [a, x, y], [" read ", " partial read ", " partial read write "], [1, 1, 1],
                        n, 5)
            np.testing.assert_array_equal(y, 2 * x + 1)
        ranges, rem = acc.ranges(5)
        assert sum(ranges) + rem == n
        acc.dispose()
    finally:
        for s in servers:
            s.dispose()
