"""NetworkBuffer codec round-trips (reference layout, NetworkBuffer.cs:32-45)
and checkpoint/resume of arrays + balancer state."""
import struct

import numpy as np
import pytest

import cekirdekler_amd as ck
from cekirdekler_amd.utils import checkpoint
from cekirdekler_amd.utils.netbuf import COMPUTE, NetworkBuffer, TYPE_FLOAT


def test_header_layout():
    nb = NetworkBuffer(COMPUTE)
    nb.add_array(np.arange(4, dtype=np.int32), 7)
    b = nb.to_bytes()
    assert b[:8] == b"Cekirdek" and b[8] == 0
    total, cmd = struct.unpack_from("<ii", b, 9)
    assert total == len(b) == 17 + 9 + 16 and cmd == COMPUTE
    assert b[17] == 2  # int32 record type


@pytest.mark.parametrize("dtype", [np.uint8, np.uint16, np.int32, np.float32, np.int64, np.float64, np.bool_])
def test_roundtrip_types(dtype):
    a = (np.arange(37) % 5).astype(dtype)
    nb = NetworkBuffer(5)
    nb.add_array(a, 123)
    cmd, recs = NetworkBuffer.parse(nb.to_bytes())
    assert cmd == 5 and len(recs) == 1
    np.testing.assert_array_equal(recs[0].data, a)
    assert recs[0].hash == 123 and recs[0].length == 37


def test_partial_float_record():
    a = np.arange(64, dtype=np.float32)
    nb = NetworkBuffer(COMPUTE)
    nb.add_array(a, -5, ref=4, range_=6, epw=2)
    nb.add_string("kernel names", 9)
    cmd, recs = NetworkBuffer.parse(nb.to_bytes())
    r = recs[0]
    # element units on the wire (reference addArray(float[]) multiplies by epw)
    assert r.type == TYPE_FLOAT and r.partial and r.ref == 8 and r.range == 12 and r.hash == -5
    np.testing.assert_array_equal(r.data, a[8:20])
    assert NetworkBuffer.record_string(recs[1]) == "kernel names"
    out = np.zeros(64, np.float32)
    r.scatter_into(out)
    np.testing.assert_array_equal(out[8:20], a[8:20])
    assert not out[:8].any() and not out[20:].any()


def test_partial_epw2_then_trailing_int_record():
    """with epw > 1 the parser must consume the whole payload,
    or every later record is misparsed."""
    a = np.arange(100, dtype=np.float32)
    nb = NetworkBuffer(COMPUTE)
    nb.add_array(a, 1, ref=3, range_=5, epw=4)      # elements [12, 32)
    nb.add_ints([7, 8, 9], 2)
    nb.add_array(a, 3, 0, 0, 4)                      # header only
    nb.add_ints([42], 4)
    cmd, recs = NetworkBuffer.parse(nb.to_bytes())
    assert [r.hash for r in recs] == [1, 2, 3, 4]
    np.testing.assert_array_equal(recs[0].data, a[12:32])
    np.testing.assert_array_equal(recs[1].data, [7, 8, 9])
    assert recs[2].partial and recs[2].range == 0 and len(recs[2].data) == 0 and recs[2].length == 100
    assert int(recs[3].data[0]) == 42


def _rec(t, h, payload: bytes, n: int, ref=None, rng=None) -> bytes:
    """One record built straight from the layout comment NetworkBuffer.cs:
    36-44: e (u8 type) h (i32 hash) s (i32 length) [r m] (float) d."""
    b = struct.pack("<Bii", t, h, n)
    if t == 3:
        b += struct.pack("<ii", ref, rng)
    return b + payload


def _buf(cmd: int, records) -> bytes:
    body = b"".join(records)
    return b"Cekirdek" + bytes([0]) + struct.pack("<ii", 17 + len(body), cmd) + body


def _u16(s: str) -> bytes:
    return s.encode("utf-16-le")


def test_golden_setup_bytes():
    from cekirdekler_amd.parallel.cluster import setup_message

    got = setup_message("gpu", "K", ["k1", "k2"], 64, -1, True, 3).to_bytes()
    want = _buf(0, [_rec(1, 0, _u16("gpu"), 3), _rec(1, 0, _u16("K"), 1), _rec(1, 0, _u16("k1 k2"), 5),
                    _rec(2, 0, struct.pack("<i", 64), 1), _rec(2, 0, struct.pack("<i", -1), 1),
                    _rec(6, 0, b"\x01", 1), _rec(2, 0, struct.pack("<i", 3), 1)])
    assert got == want


def test_golden_compute_and_answer_bytes():
    from cekirdekler_amd.parallel.cluster import answer_message, compute_message

    a = np.array([2.5], np.float32)                  # read
    x = np.arange(16, dtype=np.float32)              # partial read, epw 2
    y = np.arange(16, dtype=np.float32) + 100        # write only
    rws = ["read", "partial read", "write"]
    got = compute_message("saxpy", 1, "", [a, x, y], [11, 12, 13], rws, [1, 2, 2], 4, 7, 2,
                          False, 4, True).to_bytes()
    want = _buf(1, [
        _rec(1, 0, _u16("saxpy"), 5), _rec(2, 0, struct.pack("<i", 1), 1), _rec(1, 0, b"", 0),
        _rec(2, 0, struct.pack("<i", 3), 1),
        _rec(3, 11, a.tobytes(), 1, 0, -1),             # whole array: range -1
        _rec(3, 12, x[4:12].tobytes(), 16, 4, 8),       # ref·epw = 4, range·epw = 8 elements
        _rec(3, 13, b"", 16, 0, 0),                     # header only
        _rec(1, 0, _u16("read"), 4), _rec(1, 0, _u16("partial read"), 12), _rec(1, 0, _u16("write"), 5),
        _rec(2, 0, struct.pack("<3i", 1, 2, 2), 3), _rec(2, 0, struct.pack("<i", 4), 1),
        _rec(2, 0, struct.pack("<i", 7), 1), _rec(2, 0, struct.pack("<i", 2), 1),
        _rec(6, 0, b"\x00", 1), _rec(2, 0, struct.pack("<i", 4), 1), _rec(6, 0, b"\x01", 1)])
    assert got == want
    ans = answer_message([a, x, y], [11, 12, 13], rws, [1, 2, 2], 4, 2).to_bytes()
    want_ans = _buf(5, [_rec(3, 11, b"", 1, 0, 0), _rec(3, 12, b"", 16, 0, 0),
                        _rec(3, 13, y[4:12].tobytes(), 16, 4, 8)])
    assert ans == want_ans


def test_checkpoint_roundtrip_restores_balancer(tmp_path):
    src = "__global__ void inc(float* x) { x[get_global_id(0)] += 1.0f; }"
    cpu = ck.ClPlatforms.all().cpus(True)
    cr = ck.ClNumberCruncher(cpu + cpu, src)
    cr.set_time_scale(1, 4.0)
    x = ck.ClArray(np.zeros(1 << 14, np.float32))
    for _ in range(12):
        x.compute(cr, 3, "inc", 1 << 14, 256)
    before = cr.ranges(3)
    path = str(tmp_path / "state.cek")
    n = checkpoint.save(path, {"x": x}, cr)
    assert n > 0
    cr2 = ck.ClNumberCruncher(cpu + cpu, src)
    x2 = ck.ClArray(np.zeros(1 << 14, np.float32))
    out = checkpoint.load(path, {"x": x2}, cr2)
    np.testing.assert_array_equal(x2.array, 12.0)
    np.testing.assert_array_equal(out["x"], 12.0)
    assert cr2.ranges(3) == before
    cr2.set_time_scale(1, 4.0)
    x2.compute(cr2, 3, "inc", 1 << 14, 256)  # continues from the restored split
    assert abs(cr2.ranges(3)[0] - before[0]) <= 0.1 * (1 << 14)
