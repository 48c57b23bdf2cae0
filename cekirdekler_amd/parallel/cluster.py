"""Multi-node layer over TCP (reference "pre-alpha" cluster add-on:
ClusterAccelerator.cs, ClusterLoadBalancer.cs, ClCruncherServer(.Thread).cs,
ClCruncherClient.cs, NetworkBuffer.cs, IHesapNode.cs).

* :class:`ClCruncherServer` — TCP listener; one thread per client hosting a
  :class:`~cekirdekler_amd.cruncher.Cores` built from the client's SETUP.
* :class:`ClCruncherClient` — SETUP / COMPUTE / DISPOSE / CONTROL /
  NUM_DEVICES / STOP over the byte-compatible :mod:`netbuf` framing (the
  same record order as the reference server thread,
  ClCruncherServerThread.cs:113-248).
* :class:`ClusterAccelerator` — node-level range split with the reference's
  cluster balancer (LCM-of-steps equal split, then ``t + 0.3·(p − t)``); the
  local "mainframe" node computes the remainder (ClusterAccelerator.cs:
  170-355).  Node discovery: explicit ``host:port`` list, or a probe of
  candidate addresses with the CONTROL handshake (the reference's ping sweep
  of 192.168.1.x, :77-154, generalised to a given candidate list).

Intra-node scaling on MI355X is the job of :mod:`distributed` (RCCL/xGMI);
this layer is the TCP control+data plane between nodes.
"""
from __future__ import annotations

import socket
import struct
import threading
from dataclasses import dataclass
import time
from typing import List, Optional, Sequence

import numpy as np

from ..utils import netbuf as nbm
from ..utils.netbuf import NetworkBuffer
from .balancer import ClusterLoadBalancer

CHUNK = 8 * 1024  # reference receiveSendBufferSize


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        part = sock.recv(min(n - len(buf), 1 << 20))
        if not part:
            raise ConnectionError("connection closed")
        buf += part
    return bytes(buf)


def recv_message(sock: socket.socket) -> bytes:
    head = _recv_exact(sock, nbm.HEADER)
    total = NetworkBuffer.read_length(head)
    return head + _recv_exact(sock, total - nbm.HEADER)


def send_message(sock: socket.socket, nb: NetworkBuffer) -> None:
    sock.sendall(nb.to_bytes())


def _as_np(a):
    return a.array if hasattr(a, "array") else np.asarray(a)


class IComputeNode:
    """Node abstraction (reference IHesapNode.cs:29-59)."""

    def setup_nodes(self, *a, **k):
        raise NotImplementedError

    def compute(self, *a, **k):
        raise NotImplementedError

    def compute_timing(self) -> float:
        raise NotImplementedError

    def dispose(self) -> None:
        raise NotImplementedError


# --------------------------------------------------------------------------- server


class ClCruncherServerThread(threading.Thread):
    def __init__(self, server: "ClCruncherServer", conn: socket.socket, addr):
        super().__init__(daemon=True)
        self.server, self.conn, self.addr = server, conn, addr
        self.cores = None
        self.arrays = {}  # hash -> numpy array (persistent per client, like d0)

    def run(self) -> None:
        from ..cruncher import Cores

        try:
            while not self.server._stopping:
                msg = recv_message(self.conn)
                cmd, recs = NetworkBuffer.parse(msg)
                if cmd == nbm.SETUP:
                    types = NetworkBuffer.record_string(recs[0])
                    src = NetworkBuffer.record_string(recs[1])
                    names = NetworkBuffer.record_string(recs[2]).split()
                    local, ngpu = int(recs[3].data[0]), int(recs[4].data[0])
                    stream, maxcpu = bool(recs[5].data[0]), int(recs[6].data[0])
                    try:
                        self.cores = Cores(types, src, names, False, local, ngpu, stream, maxcpu)
                        ok = self.cores.cruncher.error_code() == 0
                    except Exception as e:  # noqa: BLE001
                        ok, err = False, str(e)
                    ans = NetworkBuffer(nbm.ANSWER_SUCCESS if ok else nbm.ANSWER_ERROR)
                    if not ok:
                        ans.add_string(self.cores.cruncher.error_message() if self.cores else err)
                    send_message(self.conn, ans)
                elif cmd == nbm.COMPUTE:
                    send_message(self.conn, self._compute(recs))
                elif cmd == nbm.DISPOSE:
                    if self.cores:
                        self.cores.dispose()
                    self.cores = None
                    send_message(self.conn, NetworkBuffer(nbm.ANSWER_DELETED))
                elif cmd == nbm.SERVER_CONTROL:
                    send_message(self.conn, NetworkBuffer(nbm.ANSWER_CONTROL))
                elif cmd == nbm.SERVER_NUMBER_OF_DEVICES:
                    ans = NetworkBuffer(nbm.ANSWER_NUMBER_OF_DEVICES)
                    ans.add_ints([self.cores.number_of_devices if self.cores else 0])
                    send_message(self.conn, ans)
                elif cmd == nbm.SERVER_STOP:
                    send_message(self.conn, NetworkBuffer(nbm.ANSWER_STOPPED))
                    self.server._stopping = True
                    break
        except (ConnectionError, OSError):
            pass
        finally:
            try:
                self.conn.close()
            except OSError:
                pass
            if self.cores:
                self.cores.dispose()

    def _compute(self, recs) -> NetworkBuffer:
        names = NetworkBuffer.record_string(recs[0])
        steps = int(recs[1].data[0])
        step_fn = NetworkBuffer.record_string(recs[2])
        n = int(recs[3].data[0])
        arr_recs = recs[4:4 + n]
        rws = [NetworkBuffer.record_string(recs[4 + n + i]) for i in range(n)]
        epw = [int(x) for x in recs[4 + 2 * n].data]
        G = int(recs[5 + 2 * n].data[0])
        cid = int(recs[6 + 2 * n].data[0])
        off = int(recs[7 + 2 * n].data[0])
        pipe = bool(recs[8 + 2 * n].data[0])
        blobs = int(recs[9 + 2 * n].data[0])
        ptype = bool(recs[10 + 2 * n].data[0])
        arrays = []
        for r, e in zip(arr_recs, epw):
            a = self.arrays.get(r.hash)
            if a is None or len(a) != r.length or a.dtype != r.data.dtype.newbyteorder("="):
                a = np.zeros(r.length, r.data.dtype.newbyteorder("="))
                self.arrays[r.hash] = a
            r.scatter_into(a)
            arrays.append(a)
        try:
            # ranges are absolute: the node computes [off, off+G) of the global range
            self.cores.compute(names, steps, step_fn, arrays, rws, epw, G, cid, off, pipe, blobs, ptype)
        except Exception as e:  # noqa: BLE001
            err = NetworkBuffer(nbm.ANSWER_ERROR)
            err.add_string(str(e))
            return err
        return answer_message(arrays, [r.hash for r in arr_recs], rws, epw, G, off)


def answer_message(arrays, hashes, read_writes, epw, global_range: int, global_offset: int) -> NetworkBuffer:
    """ANSWER_COMPUTE_COMPLETE (reference ClCruncherServerThread.cs:192-210):
    float arrays return the node's slice ``[off·e, (off+G)·e)`` as a partial
    record; other types return whole.  Float arrays the kernel does not
    write come back as header-only partial records (range 0)."""
    ans = NetworkBuffer(nbm.ANSWER_COMPUTE_COMPLETE)
    for a, h, rw, e in zip(arrays, hashes, read_writes, epw):
        if a.dtype == np.float32:
            if "write" in rw.split():
                ans.add_array(a, h, global_offset, global_range, e)
            else:
                ans.add_array(a, h, 0, 0, e)
        else:
            ans.add_array(a, h)
    return ans


class ClCruncherServer:
    """TCP compute server (reference ClCruncherServer.cs:31-152)."""

    def __init__(self, port: int = 50000, ip: str = "127.0.0.1", max_clients: int = 8):
        self.port, self.ip, self.max_clients = port, ip, max_clients
        self._sock: Optional[socket.socket] = None
        self._thread: Optional[threading.Thread] = None
        self._clients: List[ClCruncherServerThread] = []
        self._stopping = False

    def start(self) -> "ClCruncherServer":
        s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        s.bind((self.ip, self.port))
        s.listen(self.max_clients)
        s.settimeout(0.2)
        self.port = s.getsockname()[1]
        self._sock = s
        self._stopping = False
        self._thread = threading.Thread(target=self._accept_loop, daemon=True)
        self._thread.start()
        return self

    def _accept_loop(self) -> None:
        while not self._stopping:
            try:
                conn, addr = self._sock.accept()
            except socket.timeout:
                continue
            except OSError:
                break
            conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            t = ClCruncherServerThread(self, conn, addr)
            self._clients.append(t)
            t.start()

    def wait(self, timeout: Optional[float] = None) -> None:
        if self._thread:
            self._thread.join(timeout)

    continue_from_last_wait = wait

    def stop(self) -> None:
        self._stopping = True
        if self._sock:
            try:
                self._sock.close()
            except OSError:
                pass
        if self._thread:
            self._thread.join(2.0)

    def dispose(self) -> None:
        self.stop()
        for c in self._clients:
            try:
                c.conn.close()
            except OSError:
                pass


# --------------------------------------------------------------------------- client


def setup_message(device_types: str, kernels: str, kernel_names, local_range: int = 256, num_gpus: int = -1,
                  stream: bool = True, max_cpu: int = -1) -> NetworkBuffer:
    """SETUP: device types, kernel source and names (UTF-16 char records),
    local range and GPU count (int), stream (bool), max CPU (int) — the
    record order of ClCruncherClient.cs:121-153."""
    nb = NetworkBuffer(nbm.SETUP)
    nb.add_string(device_types)
    nb.add_string(kernels)
    nb.add_string(" ".join(kernel_names) if not isinstance(kernel_names, str) else kernel_names)
    nb.add_ints([local_range])
    nb.add_ints([num_gpus])
    nb.add_array(np.array([stream], np.bool_), 0)
    nb.add_ints([max_cpu])
    return nb


def compute_message(kernel_names: str, steps: int, step_fn: str, arrays, hashes, read_writes, epw,
                    global_range: int, compute_id: int, global_offset: int = 0, pipeline: bool = False,
                    blobs: int = 4, pipeline_type: bool = True) -> NetworkBuffer:
    """COMPUTE (ClCruncherClient.cs:155-256): names, steps, step function,
    array count, the array records, one read/write string per array, then
    elements-per-work-item, global range, compute id, offset, pipeline flag,
    blob count and pipeline type.

    Array records: ``partial`` float arrays carry the node's slice and
    ``read`` arrays carry the whole array, as the reference sends them.  The
    reference client omits every other array, which its own server cannot
    parse (it indexes the records by position, ClCruncherServerThread.cs:
    147-175, so the read/write strings shift).  Here such a float array is a
    header-only partial record (range 0: hash and length, no payload), which
    the reference parser reads as an empty copy; a non-float one, which has
    no range field in the layout, is sent whole."""
    nb = NetworkBuffer(nbm.COMPUTE)
    nb.add_string(kernel_names)
    nb.add_ints([steps])
    nb.add_string(step_fn or "")
    nb.add_ints([len(arrays)])
    for a, h, rw, e in zip(arrays, hashes, read_writes, epw):
        toks = rw.split()
        if a.dtype == np.float32 and "partial" in toks:
            nb.add_array(a, h, global_offset, global_range, e)
        elif "read" in toks or a.dtype != np.float32:
            nb.add_array(a, h)
        else:
            nb.add_array(a, h, 0, 0, e)
    for rw in read_writes:
        nb.add_string(rw)
    nb.add_ints(list(epw))
    nb.add_ints([global_range])
    nb.add_ints([compute_id])
    nb.add_ints([global_offset])
    nb.add_array(np.array([pipeline], np.bool_), 0)
    nb.add_ints([blobs])
    nb.add_array(np.array([pipeline_type], np.bool_), 0)
    return nb


class ClCruncherClient:
    """Client of one compute server (reference ClCruncherClient.cs:29-325)."""

    def __init__(self, port: int = 50000, ip: str = "127.0.0.1", timeout: float = 30.0):
        self.ip, self.port = ip, port
        self.exception: Optional[Exception] = None
        self.sock = socket.create_connection((ip, port), timeout=timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._hash = {}

    def _rpc(self, nb: NetworkBuffer):
        send_message(self.sock, nb)
        return NetworkBuffer.parse(recv_message(self.sock))

    def net_setup(self, device_types: str, kernels: str, kernel_names, local_range: int = 256,
                  num_gpus: int = -1, stream: bool = True, max_cpu: int = -1) -> bool:
        cmd, recs = self._rpc(setup_message(device_types, kernels, kernel_names, local_range, num_gpus,
                                            stream, max_cpu))
        if cmd != nbm.ANSWER_SUCCESS:
            raise RuntimeError("server setup failed: " + (NetworkBuffer.record_string(recs[0]) if recs else ""))
        return True

    netSetup = net_setup

    def compute(self, kernel_names: str, steps: int, step_fn: str, arrays: Sequence, read_writes: Sequence[str],
                epw: Sequence[int], global_range: int, compute_id: int, global_offset: int = 0,
                pipeline: bool = False, blobs: int = 4, pipeline_type: bool = True) -> float:
        """Runs [global_offset, global_offset+global_range) on the server and
        writes the returned slices into ``arrays``.  Returns wall ms."""
        t0 = time.perf_counter()
        nps = [_as_np(a) for a in arrays]
        hashes = [self._hash.setdefault(id(a), len(self._hash) + 1) for a in nps]
        nb = compute_message(kernel_names, steps, step_fn, nps, hashes, read_writes, epw, global_range,
                             compute_id, global_offset, pipeline, blobs, pipeline_type)
        cmd, recs = self._rpc(nb)
        if cmd == nbm.ANSWER_ERROR:
            raise RuntimeError("server compute failed: " + NetworkBuffer.record_string(recs[0]))
        for a, r, rw in zip(nps, recs, read_writes):
            if r.partial or "write" in rw.split():
                r.scatter_into(a)
        return (time.perf_counter() - t0) * 1e3

    def control(self) -> bool:
        try:
            cmd, _ = self._rpc(NetworkBuffer(nbm.SERVER_CONTROL))
            return cmd == nbm.ANSWER_CONTROL
        except (OSError, ConnectionError) as e:
            self.exception = e
            return False

    def num_devices(self) -> int:
        cmd, recs = self._rpc(NetworkBuffer(nbm.SERVER_NUMBER_OF_DEVICES))
        return int(recs[0].data[0]) if recs else 0

    numDevices = num_devices

    def stop(self) -> None:
        try:
            self._rpc(NetworkBuffer(nbm.SERVER_STOP))
        except (OSError, ConnectionError):
            pass

    def dispose(self) -> None:
        try:
            self._rpc(NetworkBuffer(nbm.DISPOSE))
        except (OSError, ConnectionError):
            pass
        try:
            self.sock.close()
        except OSError:
            pass


# --------------------------------------------------------------------------- accelerator


@dataclass
class ServerInfoSimple:
    """One discovered compute server (ClusterAccelerator.ServerInfoSimple,
    ClusterAccelerator.cs:41-47): the reference rates a server by
    1 / (0.1 + ping round trip in ms); here the round trip is the CONTROL
    handshake's."""
    port: int
    ip_string: str
    name_of_server: str = ""
    round_trip_performance: float = 0.0

    ipString = property(lambda self: self.ip_string)
    nameOfServer = property(lambda self: self.name_of_server)
    roundTripPerformance = property(lambda self: self.round_trip_performance)


def find_servers(candidates: Sequence[str], ports: Sequence[int], timeout: float = 0.3,
                 infos: Optional[List["ServerInfoSimple"]] = None) -> List[tuple]:
    """Probe ``host`` × ``port`` candidates with the CONTROL handshake, in
    parallel (the reference pings then tests each address from a
    ``Parallel.For``, ClusterAccelerator.cs:77-154).  Returns the answering
    ``(host, port)`` pairs in candidate order."""
    pairs = [(h, p) for p in ports for h in candidates]
    ok = [False] * len(pairs)
    rtt = [0.0] * len(pairs)

    def probe(i):
        host, port = pairs[i]
        try:
            c = ClCruncherClient(port, host, timeout=timeout)
        except OSError:
            return
        try:
            t0 = time.perf_counter()
            ok[i] = c.control()
            rtt[i] = (time.perf_counter() - t0) * 1e3
        finally:
            c.sock.close()

    threads = [threading.Thread(target=probe, args=(i,), daemon=True) for i in range(len(pairs))]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if infos is not None:
        infos.extend(ServerInfoSimple(p, h, h, 1.0 / (0.1 + r)) for (h, p), good, r in zip(pairs, ok, rtt) if good)
    return [pr for pr, good in zip(pairs, ok) if good]


def parse_cluster_devices(device_types: str) -> dict:
    """The reference's cluster device string (ClusterAccelerator.cs:364-443),
    e.g. ``"gpu cluster:50000,50001 fast-search node0_g"``:

    * ``cluster:P[,P...]`` — server ports to search (required);
    * ``fast-search`` — probe only the first 9 addresses of the sweep;
    * ``node0_g`` / ``node0_c`` — the local mainframe node computes on the
      GPU / the CPU (none otherwise);
    * ``gpu`` / ``cpu`` / ``acc`` anywhere in the string — the device types
      every server is set up with (the mainframe tokens count, as in the
      reference's substring test)."""
    s = device_types.lower()
    if "cluster:" not in s:
        raise ValueError("cluster device string needs 'cluster:PORT[,PORT]'")
    tail = s.split("cluster:", 1)[1].strip().split("port")[0].strip()
    ports = [int(p) for p in tail.split()[0].split(",") if p.strip()] if tail else []
    if not ports:
        raise ValueError("cluster device string needs at least one port after 'cluster:'")
    mainframe = "gpu" if "node0_g" in s else ("cpu" if "node0_c" in s else None)
    server = "".join(t for t in ("gpu", "cpu", "acc") if t in s)
    return {"ports": ports, "fast_search": "fast-search" in s, "mainframe": mainframe, "server_devices": server}


def sweep_candidates(fast: bool) -> List[str]:
    """Addresses the discovery sweep probes: the loopback, plus
    ``<prefix>1 .. <prefix>254`` (``fast``: 1..9) when ``CEK_CLUSTER_SUBNET``
    names a prefix such as ``192.168.1.`` (the reference's fixed LAN,
    ClusterAccelerator.cs:80-86), plus any hosts in ``CEK_CLUSTER_HOSTS``
    (comma separated)."""
    import os

    out = ["127.0.0.1"]
    prefix = os.environ.get("CEK_CLUSTER_SUBNET", "")
    if prefix:
        out += [f"{prefix}{i}" for i in range(1, 10 if fast else 255)]
    out += [h.strip() for h in os.environ.get("CEK_CLUSTER_HOSTS", "").split(",") if h.strip()]
    seen = set()
    return [h for h in out if not (h in seen or seen.add(h))]


class ClusterAccelerator(IComputeNode):
    """Range split over compute servers + the local mainframe node."""

    ServerInfoSimple = ServerInfoSimple

    def __init__(self):
        self.clients: List[ClCruncherClient] = []
        self.mainframe = None
        self.balancer = ClusterLoadBalancer()
        self._state = {}
        self.last_ms: List[float] = []
        self.discovered: List[tuple] = []
        self.servers: List[ServerInfoSimple] = []  # discovery results with round-trip ratings

    def setup_nodes(self, nodes, *args, **kwargs) -> None:
        """``nodes`` is an explicit ``[(host, port), ...]`` list (then
        ``device_types, kernels, kernel_names, local_range, num_gpus, stream,
        max_cpu, mainframe_types``), or the reference's device string, which
        goes to :meth:`setup_cluster` with the reference's argument order."""
        if isinstance(nodes, str):
            return self.setup_cluster(nodes, *args, **kwargs)
        return self._setup_list(nodes, *args, **kwargs)

    def setup_cluster(self, device_types: str, kernels: str = "", kernel_names=None, local_range: int = 256,
                      num_gpus: int = -1, stream: bool = True, max_cpu: int = -1) -> None:
        """Reference ``setupNodes(deviceTypes, kernelsString, kernelNames, L,
        nGPU, stream, maxCPU)`` (ClusterAccelerator.cs:364-443): parses
        ``device_types`` (:func:`parse_cluster_devices`), finds the servers
        on the given ports with the discovery sweep
        (:func:`sweep_candidates`), sets every server up with the string's
        device types and builds the ``node0_g``/``node0_c`` mainframe."""
        spec = parse_cluster_devices(device_types)
        self.servers = []
        self.discovered = find_servers(sweep_candidates(spec["fast_search"]), spec["ports"], infos=self.servers)
        self._setup_list(self.discovered, spec["server_devices"] or "gpu", kernels, kernel_names, local_range,
                         num_gpus, stream, max_cpu, spec["mainframe"])

    def _setup_list(self, nodes: Sequence[tuple], device_types: str, kernels: str, kernel_names=None,
                    local_range: int = 256, num_gpus: int = -1, stream: bool = True, max_cpu: int = -1,
                    mainframe_types: Optional[str] = None) -> None:
        from ..cruncher import Cores

        names = kernel_names or []
        for host, port in nodes:
            c = ClCruncherClient(port, host)
            c.net_setup(device_types, kernels, names, local_range, num_gpus, stream, max_cpu)
            self.clients.append(c)
        if mainframe_types:
            self.mainframe = Cores(mainframe_types, kernels, names, False, local_range, num_gpus, stream, max_cpu)
        self.local_range = local_range

    setupNodes = setup_nodes  # both call forms: device string or explicit (host, port) list

    def compute(self, kernel_names: str, steps: int, step_fn: str, arrays, read_writes, epw,
                global_range: int, compute_id: int, global_offset: int = 0, pipeline: bool = False,
                blobs: int = 4, pipeline_type: bool = True) -> None:
        L = self.local_range
        steps_n = [L * (blobs if pipeline else 1)] * len(self.clients)
        st = self._state.get(compute_id)
        if st is None:
            ranges, rem = self.balancer.equal_split(global_range, steps_n)
        else:
            ranges, rem = self.balancer.balance(st["ms"], global_range, st["ranges"], steps_n, st["rem"])
        offs, acc = [], global_offset
        for r in ranges:
            offs.append(acc)
            acc += r
        ms = [0.0] * len(self.clients)
        errors = []

        def node(i):
            try:
                ms[i] = self.clients[i].compute(kernel_names, steps, step_fn, arrays, read_writes, epw,
                                                ranges[i], compute_id, offs[i], pipeline, blobs, pipeline_type)
            except Exception as e:  # noqa: BLE001
                errors.append(e)

        threads = [threading.Thread(target=node, args=(i,)) for i in range(len(self.clients))]
        for t in threads:
            t.start()
        if rem > 0:
            if self.mainframe is None:
                raise RuntimeError("remainder range needs a mainframe node")
            self.mainframe.compute(kernel_names, steps, step_fn, arrays, read_writes, epw, rem, compute_id,
                                   acc, pipeline, blobs, pipeline_type)
        for t in threads:
            t.join()
        if errors:
            raise errors[0]
        self._state[compute_id] = {"ranges": ranges, "ms": ms, "rem": rem}
        self.last_ms = ms

    def ranges(self, compute_id: int):
        st = self._state.get(compute_id)
        return (list(st["ranges"]), st["rem"]) if st else None

    def compute_timing(self) -> float:
        return max(self.last_ms) if self.last_ms else 0.0

    def dispose(self) -> None:
        for c in self.clients:
            c.dispose()
        if self.mainframe:
            self.mainframe.dispose()
