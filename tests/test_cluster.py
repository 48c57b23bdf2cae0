"""Cluster layer on loopback: two compute servers + the local mainframe,
NetworkBuffer framing over TCP, node-level balancing."""
import numpy as np

from cekirdekler_amd.parallel.cluster import (ClCruncherClient, ClCruncherServer, ClusterAccelerator,
                                              find_servers)

SRC = """
__global__ void saxpy(const float* a, const float* x, float* y) {
  long long i = get_global_id(0);
  y[i] = a[0] * x[i] + y[i];
}
"""


def test_client_server_roundtrip():
    srv = ClCruncherServer(0, "127.0.0.1").start()
    try:
        c = ClCruncherClient(srv.port, "127.0.0.1")
        assert c.control()
        c.net_setup("cpu", SRC, ["saxpy"], 64)
        assert c.num_devices() == 1
        n = 4096
        a = np.array([3.0], np.float32)
        x = np.arange(n, dtype=np.float32)
        y = np.ones(n, np.float32)
        c.compute("saxpy", 1, "", [a, x, y], [" read ", " partial read ", " partial read write "], [1, 1, 1],
                  n // 2, 1, n // 2)
        np.testing.assert_array_equal(y[n // 2:], 3 * x[n // 2:] + 1)
        np.testing.assert_array_equal(y[:n // 2], 1)
        c.dispose()
    finally:
        srv.dispose()


def test_cluster_accelerator_with_mainframe():
    servers = [ClCruncherServer(0, "127.0.0.1").start() for _ in range(2)]
    try:
        nodes = find_servers(["127.0.0.1"], [s.port for s in servers])
        assert len(nodes) == 2
        acc = ClusterAccelerator()
        acc.setup_nodes(nodes, "cpu", SRC, ["saxpy"], 64, mainframe_types="cpu")
        n = 64 * 100 + 64 * 3  # not divisible evenly: remainder goes to the mainframe
        a = np.array([2.0], np.float32)
        x = np.arange(n, dtype=np.float32)
        for it in range(4):
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
