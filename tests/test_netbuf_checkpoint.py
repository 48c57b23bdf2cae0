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
    cmd, recs = NetworkBuffer.parse(nb.to_bytes(), epws=[2])
    r = recs[0]
    assert r.type == TYPE_FLOAT and r.partial and r.ref == 4 and r.range == 6 and r.hash == -5
    np.testing.assert_array_equal(r.data, a[8:20])
    assert NetworkBuffer.record_string(recs[1]) == "kernel names"


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
