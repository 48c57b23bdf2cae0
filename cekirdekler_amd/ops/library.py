"""Registry of the AOT gfx950 kernel library (``kernels/*.hip`` →
``*.hsaco``, built by :mod:`cekirdekler_amd.build_native`).

Each entry maps a library name to its code object and exported kernel names,
in the ``prebuilt`` form accepted by :class:`ClNumberCruncher`.  Library
kernels follow the runtime launch ABI (arrays, then the hidden offset and
global size), so they are range-partitioned and load-balanced by compute()
exactly like user kernel strings.
"""
from __future__ import annotations

import os

from .._native import kernel_dir

LIBRARY = {
    # production tiles plus at most two tested alternates each (the measured
    # losers of rounds 1-2 live in git history and profiles/gemm_*.md)
    "sgemm_bf16": ["cek_sgemm_bf16_256x256", "cek_sgemm_bf16_256x256pp", "cek_sgemm_bf16_256x256pb",
                   "cek_sgemm_bf16_256x256pbr",
                   "cek_sgemm_bf16_256x128pb", "cek_sgemm_bf16_256x128pe", "cek_sgemm_bf16_128x128",
                   "cek_sgemm_bf16_256x256pp_sk", "cek_sgemm_bf16_256x256pb_sk",
                   "cek_sgemm_bf16_256x256pb_sw", "cek_sgemm_bf16_256x256pb_sh", "cek_sgemm_bf16_256x256pb_ss"],
    "sgemm_f32": ["cek_sgemm_f32_128x128", "cek_sgemm_f32_256x128", "cek_sgemm_f32_256x256",
                  "cek_sgemm_f32_256x256ir", "cek_sgemm_f32_256x256ib7", "cek_sgemm_f32_256x128ie",
                  "cek_sgemm_f32_256x256w", "cek_sgemm_f32_256x256g", "cek_sgemm_f32_256x256gt", "cek_sgemm_f32_256x256gh",
                  "cek_sgemm_f32_256x256g8", "cek_sgemm_f32_256x256g8t",
                  "cek_sgemm_f32_256x256g8i", "cek_sgemm_f32_256x256g8h",
                  "cek_sgemm_f32_256x256g8q"],
    "mandelbrot": ["cek_mandelbrot_f32", "cek_mandelbrot_blk8_f32", "cek_mandelbrot_blk8h_f32",
                   "cek_mandelbrot_blk8k_f32", "cek_mandelbrot_blk8m_f32", "cek_mandelbrot_blk8t_f32",
                   "cek_mandelbrot_blk8u_f32", "cek_mandelbrot_blk8r_f32",
                   "cek_mandelbrot_blk8y_f32"],
    "nbody": ["cek_nbody_f32_b2", "cek_nbody_integrate_f32_b2", "cek_nbody_energy_f32_b2",
              "cek_nbody_f32_b4", "cek_nbody_integrate_f32_b4", "cek_nbody_energy_f32_b4"],
    "reduce": ["cek_reduce_sum_f32", "cek_reduce_sum_f32_x32", "cek_reduce_sum_f32_final"],
    "stream": ["cek_saxpy_f32", "cek_copy_u8", "cek_vec_add_f32"],
}

# Array-parameter count of every library kernel.  Passed to the runtime as
# "name:arity" so a compute() whose array list does not match the kernel's
# signature is rejected on the host instead of faulting on the device.
ARITY = {
    **{k: (6 if k.endswith(("_sk", "_sw", "_sh", "_ss")) else 4) for k in LIBRARY["sgemm_bf16"]},
    **{k: 4 for k in LIBRARY["sgemm_f32"]},
    **{k: 3 for k in LIBRARY["mandelbrot"]},
    **{k: 4 for k in LIBRARY["nbody"] if "energy" not in k},
    **{k: 3 for k in LIBRARY["nbody"] if "energy" in k},
    "cek_reduce_sum_f32": 2, "cek_reduce_sum_f32_x32": 2, "cek_reduce_sum_f32_final": 3,
    "cek_saxpy_f32": 3, "cek_copy_u8": 2, "cek_vec_add_f32": 3,
}


def code_object(name: str) -> str:
    path = os.path.join(kernel_dir(), name + ".hsaco")
    src = os.path.join(kernel_dir(), name + ".hip")
    stale = os.path.exists(src) and (not os.path.exists(path) or os.path.getmtime(src) > os.path.getmtime(path))
    if stale:
        from .. import build_native

        build_native.build_kernels()
    if not os.path.exists(path):
        raise FileNotFoundError(f"kernel library {name!r} not built: {path}")
    return path


def library(*names: str):
    """``prebuilt`` entries for the given library names."""
    return [(code_object(n), [f"{k}:{ARITY[k]}" for k in LIBRARY[n]]) for n in names]
