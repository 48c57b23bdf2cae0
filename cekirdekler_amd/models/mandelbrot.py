"""Mandelbrot renderer on the AOT CDNA4 kernel (BASELINE config
"Mandelbrot 4096×4096, 1×MI355X, event-driven read/compute/write pipeline").

The image is one 1-D range of work items of ``ppw`` pixels each (4 fixed
pixels for "quad"; 8 or 16 for the wave-pooled kernels, whose waves drain a
pool of 64·ppw pixels with two pixels in flight per lane); with
``pipeline=True`` each device's slice is cut into ``blobs`` chunks whose
kernel runs overlap the previous chunks' device→host copies (the reference's
event-driven pipeline, Cores.cs:1197-1367).
"""
from __future__ import annotations

import numpy as np

from ..arrays import ClArray
from ..cruncher import PIPELINE_EVENT, ClNumberCruncher
from ..ops.library import library

FLOP_PER_ITER = 8

# kernel variants; the band kernels additionally need device and pipeline
# chunk ranges made of whole 16-row bands (see kernels/mandelbrot.hip)
BAND_ROWS = {"blk8": 8, "blk8h": 8, "blk8k": 8, "blk8m": 8, "blk8t": 8, "blk8u": 8, "blk8r": 8, "blk8y": 8}  # rows per band
BAND_KERNELS = set(BAND_ROWS)
KERNELS = {
    # name: (library kernel, pixels per work item, work-group size)
    "quad": ("cek_mandelbrot_f32", 4, 256),           # 4 fixed pixels per work item
    # 8×16 pixel block per one-wave work-group (one packed pair per lane):
    # neighbouring pixels escape at similar iterations, and a finished wave's
    # slot is refilled at once
    "blk8": ("cek_mandelbrot_blk8_f32", 2, 64),        # escape counted every iteration
    # escape checked once per 8 iterations, counted after the loop from the
    # last bounded z (5 packed instructions per iteration instead of 8)
    "blk8h": ("cek_mandelbrot_blk8h_f32", 2, 64),
    # blk8h with a 4-instruction iteration, an exactly counted first block
    # (all-exterior waves end there) and no counting pass for interior waves
    "blk8k": ("cek_mandelbrot_blk8k_f32", 2, 64),
    # blk8k with a scalar prologue, a wave exit after 4 counted iterations,
    # 16-iteration blocks later on, a uniform loop and a chunked counting pass
    "blk8m": ("cek_mandelbrot_blk8m_f32", 2, 64),
    # blk8m with 32-iteration blocks and hand-ordered instruction streams
    # (the fastest; bench.py's kernel-only number)
    "blk8t": ("cek_mandelbrot_blk8t_f32", 2, 64),
    # blk8t with each launch's bands in centre-out order (longest first for
    # views centred on the set)
    "blk8u": ("cek_mandelbrot_blk8u_f32", 2, 64),
    # blk8u with a shorter per-wave prologue (loads issued together, shifts
    # instead of scalar divisions for power-of-two widths): 51.2-51.7 % vs
    # 49.8 % of FP32 peak on one stream (profiles/r5/README.md)
    "blk8r": ("cek_mandelbrot_blk8r_f32", 2, 64),
    # blk8r without per-lane checkpoints while every lane is bounded (two z
    # pairs ping-ponged; bit-identical images): the fastest, bench.py's
    # kernel-only number (53.6-53.8 % vs 52.5-52.8 % for blk8r)
    "blk8y": ("cek_mandelbrot_blk8y_f32", 2, 64),
}


class MandelbrotRenderer:
    def __init__(self, width: int = 4096, height: int = 4096, max_iter: int = 256,
                 view=(-2.0, -1.5, 3.0, 3.0), devices=None, cruncher: ClNumberCruncher | None = None,
                 kernel: str = "blk8"):
        self.kernel, self.ppw, self.local = KERNELS[kernel]
        if (width * height) % (256 * self.ppw) or width * height >= 2 ** 31:
            raise ValueError(f"width*height must be a multiple of {256 * self.ppw} and below 2^31")
        if self.local != 256 and kernel not in BAND_KERNELS:
            raise ValueError("only the band kernels take other work-group sizes")
        # band kernels: 16-row bands, whole bands per device / pipeline chunk
        self.granularity = 0
        if kernel in BAND_KERNELS:
            rows = BAND_ROWS[kernel]
            block_w = 64 * self.ppw // rows  # pixels per wave row
            if width % block_w or height % rows:
                raise ValueError(f"{kernel} needs width % {block_w} == 0 and height % {rows} == 0")
            self.granularity = rows * width // self.ppw  # one band in work items
        x0, y0, w, h = view
        self.width, self.height, self.max_iter = width, height, max_iter
        self.cr = cruncher or ClNumberCruncher(devices, "", prebuilt=library("mandelbrot"))
        self.view = ClArray(np.array([x0, y0, w / width, h / height], np.float32))
        self.size = ClArray(np.array([width, height, max_iter, 0], np.int32))
        for a in (self.view, self.size):
            a.write = False
        # The image lives in registered (hipHostRegister) host memory, not in
        # hipHostMalloc memory: device→host copies into the latter run as
        # blit kernels on the CUs beside the render; into registered pages
        # they run on the SDMA engines (1.265 vs 1.288 ms end to end for
        # 4096², tools/mandel_e2e_probe.py).
        self.out = ClArray(np.zeros(width * height, np.int32))
        self.out.read = False
        self.out.elements_per_work_item = self.ppw
        self.global_range = width * height // self.ppw
        self._last_id = None
        self._uploaded = set()  # (compute id, view bytes, size bytes) already on the devices

    def render(self, compute_id: int = 1, pipeline: bool = True, blobs: int = 8,
               pipeline_type: bool = PIPELINE_EVENT) -> np.ndarray:
        # The view and size parameters go up only when they changed since
        # this compute id last ran (two 16-byte copies on the main stream
        # would delay the first blob's kernel, and with it the first D2H,
        # by their latency).
        params = (compute_id, self.view.array.tobytes(), self.size.array.tobytes())
        fresh = params not in self._uploaded
        self.view.read = self.size.read = fresh
        self.view.next_param(self.size, self.out).compute(
            self.cr, compute_id, self.kernel, self.global_range, self.local, 0, pipeline,
            pipeline_type, blobs, granularity=self.granularity)
        self._last_id = compute_id
        if fresh:
            base, n = self.cr._cores.global_base, self.cr._cores.num_devices
            if all(r > 0 for r in self.cr.ranges(compute_id)[base:base + n]):
                self._uploaded.add(params)  # every local device holds them now
        return self.out.array.reshape(self.height, self.width)

    def local_slice(self) -> slice:
        cid = self._last_id
        refs, rng = self.cr.references(cid), self.cr.ranges(cid)
        base = self.cr._cores.global_base
        n = self.cr._cores.num_devices
        lo = refs[base] * self.ppw
        hi = (refs[base + n - 1] + rng[base + n - 1]) * self.ppw
        return slice(lo, hi)

    def flops(self) -> float:
        """FLOPs of the pixels this process computed (8 per iteration)."""
        it = self.out.array[self.local_slice()].astype(np.int64)
        return float(FLOP_PER_ITER * (it + 1).sum())

    def reference(self, rows=None) -> np.ndarray:
        x0, y0, dx, dy = (float(v) for v in self.view.array)
        ys = np.arange(self.height if rows is None else rows, dtype=np.float32)
        xs = np.arange(self.width, dtype=np.float32)
        cr = (np.float32(x0) + xs * np.float32(dx))[None, :].repeat(len(ys), 0)
        ci = (np.float32(y0) + ys * np.float32(dy))[:, None].repeat(self.width, 1)
        zr = np.zeros_like(cr)
        zi = np.zeros_like(cr)
        n = np.full(cr.shape, self.max_iter, np.int32)
        for it in range(self.max_iter):
            zr2, zi2 = zr * zr, zi * zi
            esc = (zr2 + zi2 > 4) & (n == self.max_iter)
            n[esc] = it
            t = zr * zi
            zi = t + t + ci
            zr = zr2 - zi2 + cr
        return n
