"""Pairing of the uneven all-gather-v (RcclComm::allgatherv, csrc/dist.cpp):
the grouped point-to-point ops of every rank, built by the same native
function the RCCL path issues, must pair up exactly — every send has one
receive of the same bytes at the same offset on its peer, zero-byte slices
are skipped on both sides, and every rank ends up receiving every other
rank's non-empty slice once.  Checked for world sizes 2..8 (the 8-GPU node
the driver runs), including empty ranges."""
import collections
import itertools
import random

import pytest

from cekirdekler_amd._native import cek


def _layouts(world):
    rng = random.Random(world)
    yield [4096] * world  # equal (the ring all-gather path normally takes this)
    for _ in range(6):
        sizes = [rng.choice([0, 0, 256, 4096, 12288, 65536]) for _ in range(world)]
        yield sizes
    yield [0] * (world - 1) + [1 << 20]  # one rank holds everything
    yield [1 << 20] + [0] * (world - 1)


@pytest.mark.parametrize("world", range(2, 9))
def test_allgatherv_plan_pairs_every_send(world):
    for sizes in _layouts(world):
        offsets = list(itertools.accumulate([0] + sizes[:-1]))
        plans = {r: cek.allgatherv_plan(r, world, offsets, sizes) for r in range(world)}
        sends = collections.Counter()
        recvs = collections.Counter()
        for r, plan in plans.items():
            for kind, peer, off, nbytes in plan:
                assert peer != r and 0 <= peer < world
                assert nbytes > 0, "zero-byte ops must be skipped"
                if kind == "send":
                    assert (off, nbytes) == (offsets[r], sizes[r])  # a rank only sends its own slice
                    sends[(r, peer, off, nbytes)] += 1
                else:
                    assert (off, nbytes) == (offsets[peer], sizes[peer])
                    recvs[(peer, r, off, nbytes)] += 1
        assert sends == recvs, (sizes, sends - recvs, recvs - sends)
        assert all(v == 1 for v in sends.values())
        # every rank receives every other rank's non-empty slice exactly once
        for r in range(world):
            got = sorted(peer for kind, peer, _, _ in plans[r] if kind == "recv")
            assert got == [p for p in range(world) if p != r and sizes[p] > 0]


def test_allgatherv_plan_step_order_is_a_shift():
    """Step k of every rank pairs rank r's send with rank r+k's receive, so
    the k-th ops of all ranks form one permutation (no link carries two
    slices in one step)."""
    world = 8
    sizes = [1024] * world
    offsets = [1024 * r for r in range(world)]
    for k in range(1, world):
        targets = [cek.allgatherv_plan(r, world, offsets, sizes)[2 * (k - 1)][1] for r in range(world)]
        assert sorted(targets) == list(range(world))
        assert targets == [(r + k) % world for r in range(world)]


def test_allgatherv_plan_rejects_bad_shapes():
    with pytest.raises(Exception):
        cek.allgatherv_plan(2, 2, [0, 1], [1, 1])
    with pytest.raises(Exception):
        cek.allgatherv_plan(0, 3, [0, 1], [1, 1])
