"""Load balancers.

* :func:`load_balance` / :func:`initial_split` — thin wrappers over the
  native implementation of the reference law (HelperFunctions.cs:190-280),
  which the scheduler runs per compute id.
* :func:`load_balance_py` — an independent pure-Python transcription of the
  same law, used by the tests to pin the native one.
* :class:`ClusterLoadBalancer` — node-level balancing for the cluster layer
  (ClusterLoadBalancer.cs:143-349): equal split in units of the LCM of the
  node steps, then ``t + 0.3·(p − t)`` snapped to each node's step; the
  remainder runs on the local "mainframe" node.
* :func:`convergence_iters` — the "load-balance iters" metric: computes until
  every share stays within a tolerance of its steady state.
"""
from __future__ import annotations

import math
from functools import reduce
from typing import Optional, List, Sequence, Tuple

from .._native import cek

HISTORY_DEPTH = 10


def load_balance(bench: Sequence[float], smooth: bool, history: List[List[float]], total: int,
                 ranges: Sequence[int], step: int) -> Tuple[List[int], List[List[float]]]:
    r, h = cek.load_balance(list(map(float, bench)), bool(smooth), history, int(total),
                            list(map(int, ranges)), int(step))
    return list(r), [list(x) for x in h]


def initial_split(devices: int, smooth: bool, history: List[List[float]], total: int,
                  step: int) -> Tuple[List[int], List[List[float]]]:
    r, h = cek.initial_split(int(devices), bool(smooth), history, int(total), int(step))
    return list(r), [list(x) for x in h]


def empty_history(devices: int) -> List[List[float]]:
    return [[0.0] * devices for _ in range(HISTORY_DEPTH)]


def _trunc(x: float) -> int:
    return int(math.trunc(x))


def load_balance_py(bench, smooth, history, total, ranges, step):
    """Pure-Python transcription of HelperFunctions.loadBalance."""
    n = len(ranges)
    ranges = list(ranges)
    history = [list(h) for h in history]
    total_bench = sum(bench) + 0.01 * n
    thr = [(total_bench / (bench[i] + 0.01)) * (ranges[i] + 1) for i in range(n)]
    total_thr = sum(thr)
    if total_thr <= 0.0000001:
        total_thr = 0.01
    norm = [0.0] * n
    if smooth:
        norm = [t / total_thr for t in thr]
        history = history[1:] + [norm]
        norm = [sum(h[i] for h in history) / len(history) for i in range(n)]
    tmp = [0] * n
    for i in range(n):
        p = norm[i] if (smooth and history[0][0] > 0.00001) else thr[i] / total_thr
        if ranges[i] != 0:
            tmp[i] = ranges[i] - _trunc((ranges[i] - total * p) * 0.3)
        else:
            tmp[i] = _trunc(total * (total_bench / (bench[i] + 0.01)) / total_thr)
    for i in range(n):
        rem = int(math.fmod(tmp[i], step))
        ranges[i] = tmp[i] - rem if rem < step // 2 else tmp[i] + (step - rem)
    while sum(ranges) > total:
        ranges[ranges.index(max(ranges))] -= step
    while sum(ranges) < total:
        ranges[ranges.index(max(ranges))] += step
    return ranges, history


def steady_share(shares: Sequence[float], tail: int = 10) -> float:
    """Steady state of a share trajectory: the median of its last ``tail``
    calls (one noisy final call cannot move it)."""
    last = sorted(shares[-max(1, int(tail)):])
    n = len(last)
    return last[n // 2] if n % 2 else 0.5 * (last[n // 2 - 1] + last[n // 2])


def convergence_iters(shares: Sequence[float], tol: float = 0.05, tail: int = 10) -> int:
    """The "load-balance iters" metric: 1-based index of the first call whose
    share is within ``tol`` (relative) of the steady state
    (:func:`steady_share`) and after which the share stays there — isolated
    timing outliers allowed, at most one per ten later calls (at least one):
    a single late blip, which the damped law absorbs in a few calls, is
    noise on the host clock, not a lack of convergence."""
    steady = steady_share(shares, tail)
    band = tol * abs(steady)
    out = [abs(s - steady) > band for s in shares]
    for i in range(len(shares)):
        if out[i]:
            continue
        rest = len(shares) - i
        if sum(out[i:]) <= max(1, rest // 10):
            return i + 1
    return len(shares)


def measure_lb_convergence(devices, calls: int = 40, slow_device: int = 1, slowdown: float = 2.0,
                           n: int = 1 << 22, inner: int = 2048, outliers: Sequence[int] = (),
                           outlier_scale: float = 6.0, tol: float = 0.05) -> dict:
    """The bench's "load-balance iters" measurement, reusable: computes of one
    compute id on ``devices`` (two devices; device ``slow_device``'s timings
    scaled by ``slowdown``, the reference's heterogeneous pair), a
    compute-heavy kernel so each device's time is proportional to its range.
    ``outliers``: call indices whose slow-device timing is scaled by
    ``outlier_scale`` instead (an injected timing blip).  Returns the iters,
    the steady share of device 0 and the whole share trajectory."""
    from ..arrays import ClArray
    from ..cruncher import ClNumberCruncher
    import numpy as np

    src = ("__global__ void k(float* x){ long long i = get_global_id(0); float v = x[i];\n"
           f"    for (int j = 0; j < {int(inner)}; ++j) v = v * 0.999f + 1.0f; x[i] = v; }}")
    cr = ClNumberCruncher(devices, src)
    try:
        cr.cores.serial = True  # logical devices of one GPU: time each in isolation
        x = ClArray(n, np.float32)
        x.read = False
        x.write = False
        shares = []
        bad = set(int(o) for o in outliers)
        for call in range(calls):
            cr.set_time_scale(slow_device, outlier_scale if call in bad else slowdown)
            x.compute(cr, 7, "k", n, 256)
            r = cr.ranges(7)
            shares.append(r[0] / sum(r))
        return {"iters": convergence_iters(shares, tol), "steady_share_dev0": steady_share(shares),
                "tol": tol, "calls": calls, "shares": [round(s, 5) for s in shares]}
    finally:
        cr.dispose()


def simulate(speeds: Sequence[float], total: int, step: int, calls: int = 30, smooth: bool = True):
    """Run the native law against devices with fixed throughputs (items/ms);
    returns the list of range vectors per call.  Used to measure convergence
    without hardware noise."""
    d = len(speeds)
    hist = empty_history(d)
    ranges, hist = initial_split(d, smooth, hist, total, step)
    out = [list(ranges)]
    for _ in range(calls - 1):
        bench = [r / s for r, s in zip(ranges, speeds)]
        ranges, hist = load_balance(bench, smooth, hist, total, ranges, step)
        out.append(list(ranges))
    return out


# --------------------------------------------------------------------- cluster


def _gcd(a: int, b: int) -> int:
    return math.gcd(a, b) or 64


def lcm(values: Sequence[int]) -> int:
    return reduce(lambda a, b: a // _gcd(a, b) * b, values)


class ClusterLoadBalancer:
    """Node-level balancer (reference ClusterLoadBalancer)."""

    def equal_split(self, total: int, steps: Sequence[int]) -> Tuple[List[int], int]:
        """Returns (per-node ranges, remainder for the mainframe)."""
        n = len(steps)
        l = lcm(list(steps))
        layers = (total // l) // n
        if layers == 0:
            ranges = list(steps)
            return ranges, total - sum(ranges)
        ranges = [layers * l] * n
        left = total - layers * l * n
        extra = left // l
        for i in range(extra):
            ranges[i] += l
        left -= extra * l
        return ranges, left

    @staticmethod
    def _nearest(d: float, a: int, m: int) -> int:
        tmp = int(d * m)
        k = tmp // a
        if tmp - k * a >= a // 2:
            k += 1
        return max(1, k) * a

    def balance(self, ms: Sequence[float], total: int, ranges: Sequence[int], steps: Sequence[int],
                mainframe_items: int = 0) -> Tuple[List[int], int]:
        n = len(ranges)
        ms = [max(abs(t), 0.0001) for t in ms]
        perf = [ranges[i] / ms[i] for i in range(n)]
        tp = sum(perf) or 0.001
        if total - mainframe_items == 0:
            mainframe_items = 0
        out = []
        for i in range(n):
            p = perf[i] / tp
            t = ranges[i] / float(total - mainframe_items)
            out.append(self._nearest(t + 0.3 * (p - t), steps[i], total))
        s = sum(out)
        if s <= total:
            return out, total - s
        excess = s - total
        for i in range(n):
            k = max(1, excess // steps[i])
            if steps[i] * k < excess:
                k += 1
            cut = steps[i] * k
            if out[i] - cut > 0:
                out[i] -= cut
                return out, cut - excess
        return out, 0

    # ---- the reference's spellings and call shapes (ClusterLoadBalancer.cs):
    # ranges are filled in place and the mainframe's remainder is returned;
    # tmpMenziller / tmpHizlar keep the last ranges / per-node throughputs.
    tmpMenziller: Optional[List[int]] = None
    tmpHizlar: Optional[List[float]] = None

    def dengeleEsit(self, toplamMenzil: int, menziller: List[int], adim: Sequence[int]) -> int:  # noqa: N802,N803
        """Equal first split (ClusterLoadBalancer.cs:143)."""
        ranges, rem = self.equal_split(toplamMenzil, adim)
        menziller[:] = ranges
        self.tmpMenziller = list(ranges)
        return rem

    def balanceOnPerformances(self, sureler: Sequence[float], toplamMenzil: int, menziller: List[int],  # noqa: N802,N803
                              adim: Sequence[int], anaBilgisayarThread: int = 0,  # noqa: N803
                              anaBilgisayarSure: float = 0.0) -> int:  # noqa: N803
        """Damped re-split (ClusterLoadBalancer.cs:233).  Returns the
        mainframe's remainder, or -1 when an over-subscribed split could not be
        cut back on any node (the reference's return value in that case)."""
        ms = [max(abs(t), 0.0001) for t in sureler]
        self.tmpHizlar = [menziller[i] / ms[i] for i in range(len(menziller))]
        before = list(menziller)
        ranges, rem = self.balance(sureler, toplamMenzil, before, adim, anaBilgisayarThread)
        menziller[:] = ranges
        self.tmpMenziller = list(ranges)
        if rem == 0 and sum(ranges) > toplamMenzil:
            return -1
        return rem

    def sonuc(self) -> None:
        """Prints the last ranges and their sum (ClusterLoadBalancer.cs:56)."""
        if self.tmpMenziller is not None:
            print(" ".join(str(r) for r in self.tmpMenziller))
            print(sum(self.tmpMenziller))

    @staticmethod
    def obeb(a: int, b: int) -> int:
        """Greatest common divisor (ClusterLoadBalancer.cs:72)."""
        return _gcd(a, b)

    @staticmethod
    def okek(data: Sequence[int]) -> int:
        """Least common multiple of every step (ClusterLoadBalancer.cs:121)."""
        return lcm(list(data))

