"""CU partitions of one GPU as logical devices (ClDevices.cu_partitions,
cek.partition_cus).  CPU tier: the partition map itself.
The GPU tier (tests/test_gpu_features.py) checks where the work-groups of a
partitioned device actually run."""
import pytest

import cekirdekler_amd as ck
from cekirdekler_amd._native import cek


@pytest.mark.parametrize("parts", [2, 4, 8])
def test_partitions_are_disjoint_and_cover_every_cu(parts):
    ncu = 256
    sets = [set(cek.partition_cus(ncu, parts, p)) for p in range(parts)]
    assert all(len(s) == ncu // parts for s in sets)
    assert set().union(*sets) == set(range(ncu))
    assert sum(len(s) for s in sets) == ncu


@pytest.mark.parametrize("parts", [2, 4, 8])
@pytest.mark.parametrize("numbering", ["blocked", "interleaved"])
def test_every_partition_spans_every_xcd(parts, numbering):
    """Whether the CU mask numbers CUs XCD by XCD (32 per XCD) or round robin
    over the 8 XCDs, every partition gets ncu / parts / 8 CUs on every XCD:
    each logical device keeps all 8 L2s and the XCD-aware tile mappings of
    the kernels stay balanced."""
    ncu, xcds = 256, 8
    xcd = (lambda c: c // (ncu // xcds)) if numbering == "blocked" else (lambda c: c % xcds)
    for p in range(parts):
        per = [0] * xcds
        for c in cek.partition_cus(ncu, parts, p):
            per[xcd(c)] += 1
        assert per == [ncu // parts // xcds] * xcds, (p, per)


def test_partition_arguments_checked():
    with pytest.raises(Exception):
        cek.partition_cus(256, 3, 0)
    with pytest.raises(Exception):
        cek.partition_cus(256, 8, 8)


def test_cu_partitions_keep_cpu_devices():
    cpu = ck.ClPlatforms.all().cpus(True)
    assert len(cpu.cu_partitions(4)) == len(cpu)
    assert cpu.cu_partitions(4).device(0).cu_partition is None


def test_pick_crossover():
    """The measured broadcast / per-GPU upload threshold (SURVEY §5.8 item
    3): the smallest size from which the staged fan-out stays faster."""
    from cekirdekler_amd.utils.multigpu import pick_crossover

    sizes = [1, 2, 4, 8]
    assert pick_crossover(sizes, [1, 1, 1, 1], [2, 0.5, 0.5, 0.5]) == 2
    assert pick_crossover(sizes, [1, 1, 1, 1], [0.5, 2, 0.5, 0.5]) == 4  # must STAY faster
    assert pick_crossover(sizes, [1, 1, 1, 1], [0.5] * 4) == 1
    assert pick_crossover(sizes, [1, 1, 1, 1], [2, 2, 2, 2]) is None


def test_calibrate_peer_reads_needs_two_gpus():
    import cekirdekler_amd as ck

    cr = ck.ClNumberCruncher(ck.ClPlatforms.all().cpus(True), "__global__ void k(float* a) {}")
    before = cr.peer_read_min_bytes
    out = cr.calibrate_peer_reads()
    assert "skipped" in out and cr.peer_read_min_bytes == before
    cr.dispose()
