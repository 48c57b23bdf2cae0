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


def test_parse_cluster_device_string():
    from cekirdekler_amd.parallel.cluster import parse_cluster_devices

    d = parse_cluster_devices("GPU cluster:50000,50001 fast-search node0_c")
    assert d["ports"] == [50000, 50001] and d["fast_search"] and d["mainframe"] == "cpu"
    assert d["server_devices"] == "gpu"  # "node0_c" does not contain "cpu"
    d = parse_cluster_devices("cpu cluster: 4000 port node0_g")
    assert d["ports"] == [4000] and not d["fast_search"] and d["mainframe"] == "gpu"
    import pytest
    with pytest.raises(ValueError):
        parse_cluster_devices("gpu cpu")


def test_cluster_setup_by_device_string(monkeypatch):
    """Reference setupNodes(deviceTypes, ...) path: ports from the string,
    servers found by the discovery sweep (loopback + CEK_CLUSTER_HOSTS),
    mainframe from node0_c."""
    servers = [ClCruncherServer(0, "127.0.0.1").start() for _ in range(2)]
    try:
        monkeypatch.setenv("CEK_CLUSTER_HOSTS", "127.0.0.1")
        acc = ClusterAccelerator()
        ports = ",".join(str(s.port) for s in servers)
        acc.setupNodes(f"cpu cluster:{ports} fast-search node0_c", SRC, ["saxpy"], 64)
        assert sorted(acc.discovered) == sorted(("127.0.0.1", s.port) for s in servers)
        # ServerInfoSimple records (ClusterAccelerator.cs:41-47) with round-trip ratings
        assert sorted((i.ipString, i.port) for i in acc.servers) == sorted(acc.discovered)
        assert all(i.roundTripPerformance > 0 for i in acc.servers)
        assert isinstance(acc.servers[0], ClusterAccelerator.ServerInfoSimple)
        assert acc.mainframe is not None
        n = 64 * 50 + 64
        a = np.array([4.0], np.float32)
        x = np.arange(n, dtype=np.float32)
        for _ in range(3):
            y = np.ones(n, np.float32)
            acc.compute("saxpy", 1, "", [a, x, y], [" read ", " partial read ", " partial read write "], [1, 1, 1],
                        n, 2)
            np.testing.assert_array_equal(y, 4 * x + 1)
        acc.dispose()
    finally:
        for s in servers:
            s.dispose()


def test_partial_epw2_over_the_wire():
    """epw = 2 partial arrays through a server: the slice lands at element
    offset ref·epw on both sides."""
    src = """__global__ void dbl(float* y) { long long i = get_global_id(0); y[2*i] *= 2.0f; y[2*i+1] *= 3.0f; }"""
    srv = ClCruncherServer(0, "127.0.0.1").start()
    try:
        c = ClCruncherClient(srv.port, "127.0.0.1")
        c.net_setup("cpu", src, ["dbl"], 64)
        n = 256
        y = np.ones(2 * n, np.float32)
        c.compute("dbl", 1, "", [y], ["partial read write"], [2], n // 2, 1, n // 2)
        want = np.ones(2 * n, np.float32)
        want[n:][0::2] = 2.0
        want[n:][1::2] = 3.0
        np.testing.assert_array_equal(y, want)
        c.dispose()
    finally:
        srv.dispose()
