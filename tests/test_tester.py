"""The reference's in-library test suite (Tester.cs), made reachable:
the dtype × storage × device-count × pipeline × kernel-count copy matrix,
host-array behaviour, N-body vs host reference, streaming vector add."""
import pytest

import cekirdekler_amd as ck
from cekirdekler_amd.utils import tester


def test_type_matrix_cpu_logical_devices():
    cpu = ck.ClPlatforms.all().cpus(True)
    total, fails = tester.type_matrix(cpu + cpu, verbose=True)
    assert total == len(tester.MATRIX_TYPES) * 2 * 2 * 3 * 3
    assert fails == 0


def test_buffers():
    assert tester.buffers() == 0


def test_nbody_small_cpu():
    cpu = ck.ClPlatforms.all().cpus(True)
    assert tester.nbody(512, cpu + cpu, log=False, iterations=3) == 0


def test_stream_vector_add_cpu():
    assert tester.stream_c_equals_a_plus_b(1 << 16, "cpu", iterations=3) == 0


@pytest.mark.gpu
def test_type_matrix_gpu():
    g = ck.ClPlatforms.all().gpus()
    total, fails = tester.type_matrix(g[0] + g[0] if len(g) == 1 else g, verbose=True)
    assert fails == 0 and total == len(tester.MATRIX_TYPES) * 36


@pytest.mark.gpu
def test_nbody_reference_size_gpu():
    assert tester.nbody(8192, ck.ClPlatforms.all().gpus()[0:1], log=False, iterations=150) == 0


@pytest.mark.gpu
def test_stream_vector_add_cpu_gpu():
    assert tester.stream_c_equals_a_plus_b(1 << 20, "cpu gpu", iterations=10) == 0
