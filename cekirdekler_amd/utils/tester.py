"""In-library tests (reference ``Tester``, Tester.cs:29-7845), made reachable.

* :func:`type_matrix` — the reference's 252 private copy tests
  (7 dtypes × {host array, native FastArr} × {1 device, all devices} ×
  {no pipeline, event pipeline, driver pipeline} × {1, 2, 3 kernels},
  Tester.cs:32-6756; aggregated by the never-called
  ``testTypesWithFeatures``, :6758-7068).  Here bf16 is added as an 8th type
  and the global range is scaled with the device count (the reference's
  1024 items cap out at 4 devices).
* :func:`buffers` — host-array behaviour (indexing, sums, CopyFrom/CopyTo,
  native↔host switching; Tester.cs:7076-7672).
* :func:`nbody` — the O(n²) 2-D force test against a host reference,
  150 iterations through the same compute id (exercises the balancer),
  tolerance 0.01 (Tester.cs:7682-7790) — with the reference's ``fy``
  typo (it accumulates dx) fixed.
* :func:`stream_c_equals_a_plus_b` — "usage type 2" streaming vector add
  over cpu+gpu with the driver pipeline, 8 blobs (Tester.cs:7806-7843); every
  element is checked, not just element 700.
"""
from __future__ import annotations

import itertools
import time
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..arrays import BFLOAT16, ClArray, FastArr
from ..cruncher import PIPELINE_DRIVER, PIPELINE_EVENT, ClNumberCruncher, Cores
from ..hardware import ClDevices, ClPlatforms

MATRIX_TYPES = {
    "byte": (np.uint8, "unsigned char"),
    "char": (np.uint16, "unsigned short"),
    "int": (np.int32, "int"),
    "uint": (np.uint32, "unsigned int"),
    "long": (np.int64, "long long"),
    "float": (np.float32, "float"),
    "double": (np.float64, "double"),
    "bf16": (BFLOAT16, "unsigned short"),
}


def _copy_kernels(ctype: str) -> str:
    body = "{ long long i = get_global_id(0); data2[i] = data[i]; }"
    return "\n".join(f"__global__ void test{k}(const {ctype}* data, {ctype}* data2) {body}"
                     for k in ("", "2", "3"))


def matrix_cases(devices_all: bool = True):
    for tname, fast, all_dev, pipe, nk in itertools.product(
            MATRIX_TYPES, (False, True), (False, True) if devices_all else (False,),
            (None, PIPELINE_EVENT, PIPELINE_DRIVER), (1, 2, 3)):
        yield tname, fast, all_dev, pipe, nk


def matrix_case(tname: str, fast: bool, devices: ClDevices, pipe: Optional[bool], nk: int,
                cruncher_cache: Optional[Dict] = None, local: int = 64, blobs: int = 4) -> int:
    """One copy test; returns 0 on success, 1 on mismatch (reference return
    convention)."""
    dtype, ctype = MATRIX_TYPES[tname]
    key = (ctype, id(devices))
    if cruncher_cache is not None and key in cruncher_cache:
        cr = cruncher_cache[key]
    else:
        cr = ClNumberCruncher(devices, _copy_kernels(ctype))
        if cruncher_cache is not None:
            cruncher_cache[key] = cr
    D = len(devices)
    n = max(1024, local * D * (blobs if pipe is not None else 1) * 4)
    if fast:
        src = ClArray(n, dtype)
        dst = ClArray(n, dtype)
    else:
        np_dt = np.uint16 if dtype == BFLOAT16 else dtype
        src = ClArray(np.zeros(n, np_dt), dtype if dtype == BFLOAT16 else None)
        dst = ClArray(np.zeros(n, np_dt), dtype if dtype == BFLOAT16 else None)
    rng = np.random.default_rng(n + nk)
    vals = rng.integers(1, 120, n)
    src.array[:] = vals.astype(src.array.dtype)
    dst.array[:] = 0
    names = " ".join(["test", "test2", "test3"][:nk])
    if pipe is None:
        src.next_param(dst).compute(cr, 1, names, n, local)
    else:
        src.partial_read = True
        src.next_param(dst).compute(cr, 1, names, n, local, 0, True, pipe, blobs)
    return 0 if np.array_equal(src.array, dst.array) else 1


def type_matrix(devices: Optional[ClDevices] = None, verbose: bool = False) -> Tuple[int, int]:
    """Runs every matrix case; returns (cases, failures)."""
    plats = ClPlatforms.all()
    all_devs = devices if devices is not None else (plats.gpus() if len(plats.gpus()) else plats.cpus(True))
    one = all_devs[0]
    cache: Dict = {}
    fails = total = 0
    for tname, fast, all_dev, pipe, nk in matrix_cases(len(all_devs) > 1):
        devs = all_devs if all_dev else one
        r = matrix_case(tname, fast, devs, pipe, nk, cache)
        total += 1
        fails += r
        if verbose and r:
            print(f"FAIL {tname} fast={fast} all={all_dev} pipe={pipe} kernels={nk}")
    return total, fails


def buffers() -> int:
    """Host-array behaviour for every type (reference byte/char/int/.../
    longArrayOperations + buffers(), Tester.cs:7076-7672)."""
    err = 0
    for tname, (dtype, _) in MATRIX_TYPES.items():
        n = 1024
        a = ClArray(n, dtype)                 # native pinned
        b = ClArray(FastArr(n, dtype))        # explicit FastArr
        np_dt = np.uint16 if dtype == BFLOAT16 else dtype
        c = ClArray(np.zeros(n, np_dt))       # host array
        ref = (np.arange(n) % 200).astype(np_dt)
        for x in (a, b, c):
            for i in range(0, n, 97):
                x[i] = ref[i]
            x.array[:] = ref
            if int(x.array.astype(np.int64).sum()) != int(ref.astype(np.int64).sum()):
                err += 1
        rev = ref[::-1].copy()
        a.CopyFrom(rev, 0)
        out = np.zeros(n, np_dt)
        a.CopyTo(out, 0)
        err += 0 if np.array_equal(out, rev) else 1
        a.fast_arr = False                    # switch native → host keeps contents
        err += 0 if np.array_equal(a.array, rev) else 1
        a.fast_arr = True
        err += 0 if (np.array_equal(a.array, rev) and a.fast_arr) else 1
        for x in (a, b):
            x.dispose()
    return err


def nbody(n: int = 8 * 1024, devices: Optional[ClDevices] = None, stream: bool = False, log: bool = True,
          iterations: int = 150, check: bool = True, timing: Optional[list] = None) -> int:
    """2-D all-pairs forces (softening 1e-4), host reference vs device.
    With ``timing`` (a list), one untimed warm-up compute runs first and the
    wall time of the ``iterations`` computes (ms) is appended to it."""
    rng = np.random.default_rng(1234)
    x = (rng.random(n, dtype=np.float64) * 30 - 15).astype(np.float32)
    y = (rng.random(n, dtype=np.float64) * 30 - 15).astype(np.float32)
    src = f"""
    __global__ void nBody(const float* x, const float* y, float* fx, float* fy) {{
        int i = (int)get_global_id(0);
        float fx0 = 0.0f, fy0 = 0.0f;
        for (int j = 0; j < {n}; j++) {{
            float dx = x[i] - x[j];
            float dy = y[i] - y[j];
            float r = sqrtf(dx * dx + dy * dy + 0.0001f);
            float inv = 1.0f / (r * r * r);
            fx0 += dx * inv;
            fy0 += dy * inv;
        }}
        fx[i] = fx0;
        fy[i] = fy0;
    }}"""
    devices = devices if devices is not None else ClPlatforms.all().gpus()
    cr = ClNumberCruncher(devices, src)
    if cr.error_code():
        if log:
            print(cr.error_message())
        return 1
    cr.performance_feed = log
    xa, ya = ClArray(x), ClArray(y)
    xa.write = ya.write = False
    fx, fy = ClArray(np.zeros(n, np.float32)), ClArray(np.zeros(n, np.float32))
    fx.read = fy.read = False
    if timing is not None:
        xa.next_param(ya, fx, fy).compute(cr, 1, "nBody", n, 64)  # build buffers, first upload
        t0 = time.perf_counter()
    for _ in range(iterations):
        xa.next_param(ya, fx, fy).compute(cr, 1, "nBody", n, 64)
    if timing is not None:
        timing.append((time.perf_counter() - t0) * 1e3)
    if not check:
        cr.dispose()
        return 0
    # The reference compares against a float32 host loop in the same order
    # with an absolute 0.01; against a float64 reference the float32
    # summation error scales with Σ|terms| (close pairs give huge terms), so
    # the bound is 0.01 + 2e-6·Σ|terms|.
    err = 0
    for s in range(0, n, 1024):
        dx = x[s:s + 1024, None].astype(np.float64) - x[None, :]
        dy = y[s:s + 1024, None].astype(np.float64) - y[None, :]
        r = np.sqrt(dx * dx + dy * dy + 0.0001)
        inv = 1.0 / (r * r * r)
        tx, ty = dx * inv, dy * inv
        hfx, hfy = tx.sum(1), ty.sum(1)
        bx = 0.01 + 2e-6 * np.abs(tx).sum(1)
        by = 0.01 + 2e-6 * np.abs(ty).sum(1)
        bad = (np.abs(hfx - fx.array[s:s + 1024]) > bx) | (np.abs(hfy - fy.array[s:s + 1024]) > by)
        err += int(bad.sum())
    cr.dispose()
    return 1 if err else 0


def stream_c_equals_a_plus_b(n: int = 1024 * 1024, types: str = "cpu gpu", iterations: int = 10,
                             log: bool = False) -> int:
    a = ClArray(n, np.float32)
    b = np.arange(n, dtype=np.float32)
    c = ClArray(n, np.float32)
    a.array[:] = 3
    c.array[:] = 105
    cores = Cores(types, """
        __global__ void vectorAdd(const float* a, const float* b, float* c) {
            long long i = get_global_id(0);
            c[i] = a[i] + b[i];
        }""", ["vectorAdd"])
    for _ in range(iterations):
        cores.compute("vectorAdd", 0, "", [a, b, c], ["partial read", "partial read", "write"], [1, 1, 1], n, 1,
                      0, True, 8, PIPELINE_DRIVER, 256)
        if log:
            cores.performance_report(1)
    ok = np.array_equal(c.array, a.array + b)
    cores.dispose()
    return 0 if ok else 1
