"""Surface wave on mesh vertices: the reference's only application example
(Unity ``Kamera.cs:188-284``), run through the same public API.

Every frame displaces each vertex along its normal by
``0.02 · ctr · sin(40 t + 100 · |xy − xy₀|)`` (Kamera.cs:234-246).  Vertices and
normals are arrays of ``Vector3`` structs wrapped as byte arrays
(``wrapArrayOfStructs``, Kamera.cs:254-255) and the scalars travel in a
64-float argument array (Kamera.cs:256-264); the kernel is the reference's
OpenCL-C text, compiled through the dialect rewrite.  After the first frame
base vertices and normals stay on the devices (``read = False``,
Kamera.cs:271-272), so only the displaced slice moves each frame.

Differences from the reference, on purpose:

* ``elements_per_work_item = 12`` on the byte views (one 3-float struct per
  work item), so a multi-device split moves exactly each device's vertices —
  the reference leaves it at 1 and relies on whole-array reads.
* the vertex count need not be a multiple of the workgroup size: the range is
  rounded up and the kernel's ``id < arguments[4]`` guard masks the tail
  (the reference hard-codes 224·256).
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from ..arrays import ClArray
from ..cruncher import ClNumberCruncher

VERTEX = np.dtype([("x", np.float32), ("y", np.float32), ("z", np.float32)])

# Kamera.cs:234-246, verbatim semantics, OpenCL-C dialect.
WAVE_KERNEL = r"""
__kernel void waveEquation(__global float* xyz, __global float* xyzn, __global float* xyzo,
                           __global float* arguments)
{
    int threadId = get_global_id(0);
    if (threadId < arguments[4])
    {
        float dx = xyz[threadId * 3] - arguments[2];
        float dy = xyz[threadId * 3 + 1] - arguments[3];
        float t = arguments[1];
        float ctr = arguments[0];
        float wave = 0.02f * ctr * sin(40.0f * t + 100.0f * sqrt(dx * dx + dy * dy));
        xyzo[threadId * 3] = xyz[threadId * 3] + xyzn[threadId * 3] * wave;
        xyzo[threadId * 3 + 1] = xyz[threadId * 3 + 1] + xyzn[threadId * 3 + 1] * wave;
        xyzo[threadId * 3 + 2] = xyz[threadId * 3 + 2] + xyzn[threadId * 3 + 2] * wave;
    }
}
"""


def grid_mesh(nx: int = 224, ny: int = 256, extent: float = 1.0):
    """A flat nx×ny vertex grid with +z normals (the Unity plane mesh)."""
    xs = np.linspace(-extent, extent, nx, dtype=np.float32)
    ys = np.linspace(-extent, extent, ny, dtype=np.float32)
    gx, gy = np.meshgrid(xs, ys, indexing="xy")
    v = np.zeros(nx * ny, VERTEX)
    v["x"], v["y"] = gx.reshape(-1), gy.reshape(-1)
    nrm = np.zeros(nx * ny, VERTEX)
    nrm["z"] = 1.0
    return v, nrm


def wave_reference(base: np.ndarray, normals: np.ndarray, ctr: float, t: float, x0: float,
                   y0: float) -> np.ndarray:
    """float32 host version of the kernel (the reference's CPU branch,
    Kamera.cs:210-218)."""
    dx = base["x"] - np.float32(x0)
    dy = base["y"] - np.float32(y0)
    w = (np.float32(0.02) * np.float32(ctr) *
         np.sin(np.float32(40.0) * np.float32(t) + np.float32(100.0) * np.sqrt(dx * dx + dy * dy)))
    out = np.empty_like(base)
    for c in ("x", "y", "z"):
        out[c] = base[c] + normals[c] * w.astype(np.float32)
    return out


class WaveSurface:
    """Animated mesh: call :meth:`update` once per frame."""

    def __init__(self, base: np.ndarray, normals: np.ndarray, devices=None,
                 cruncher: Optional[ClNumberCruncher] = None, local: int = 64, zero_copy_output: bool = True):
        if base.dtype != VERTEX or normals.dtype != VERTEX or len(base) != len(normals):
            raise ValueError("base and normals must be equal-length VERTEX arrays")
        self.n = len(base)
        self.local = local
        self.range = -(-self.n // local) * local
        self.cr = cruncher or ClNumberCruncher(devices, WAVE_KERNEL)
        # vertex storage padded to the work range so every slice is in bounds
        self.base = np.zeros(self.range, VERTEX)
        self.base[:self.n] = base
        self.normals = np.zeros(self.range, VERTEX)
        self.normals[:self.n] = normals
        self.vertices = self.base.copy()
        self.xyz = ClArray.wrap_array_of_structs(self.base)
        self.xyzn = ClArray.wrap_array_of_structs(self.normals)
        self.xyzo = ClArray.wrap_array_of_structs(self.vertices)
        self.vertices = self.xyzo.array.view(VERTEX)   # the byte view's storage
        for a in (self.xyz, self.xyzn, self.xyzo):
            a.elements_per_work_item = VERTEX.itemsize
        self.xyz.write = self.xyzn.write = False
        self.xyzo.read = False
        # The displaced vertices are read by the host every frame: GPUs store
        # them straight into the registered host array (zero-copy over PCIe)
        # instead of a D2H copy after the kernel (0.0399 vs 0.0498 ms per
        # GPU frame, tools/wave_zc_probe.py).
        self.xyzo.zero_copy = bool(zero_copy_output)
        # the 256-byte argument block, new every frame, in pinned memory that
        # GPU kernels read in place (zero-copy): no copy command in the
        # frame's stream (0.0360 vs 0.0389 ms per GPU frame with a per-frame
        # upload, tools/wave_args_probe.py, profiles/r5/wave_args_s23.json)
        self.arguments = ClArray(64, np.float32)
        self.arguments.array[:] = 0
        self.arguments.write = False
        self.arguments.partial_read = False
        self.arguments.zero_copy = True
        self.t = 0.0
        self.ctr = 0.0
        # the per-frame constants (Kamera.cs:256-264) go in once; a frame
        # writes only ctr and t
        args = self.arguments.array
        args[2], args[3] = self.base["x"][0], self.base["y"][0]
        args[4] = self.n
        self._group = self.xyz.next_param(self.xyzn, self.xyzo, self.arguments)
        self._first = True

    def update(self, compute_id: int = 1) -> np.ndarray:
        """One frame (Kamera.cs:199-275); returns the displaced vertices."""
        if self.ctr < 0.3:
            self.ctr += 0.001
        self.t += 0.001
        args = self.arguments.array
        args[0], args[1] = self.ctr, self.t
        self._group.compute(self.cr, compute_id, "waveEquation", self.range, self.local)
        if self._first:  # base vertices and normals stay on the devices (Kamera.cs:271-272)
            self.xyzn.read = False
            self.xyz.read = False
            self._first = False
        return self.vertices[:self.n]

    def reference(self) -> np.ndarray:
        return wave_reference(self.base[:self.n], self.normals[:self.n], np.float32(self.ctr),
                              np.float32(self.t), self.base["x"][0], self.base["y"][0])


class ReferenceCpuWave:
    """The reference example's CPU-only strategy (Kamera.cs:208-218,
    ``strategy = true``): no runtime, one host thread updating the vertices
    one at a time with double-precision ``Math.Sqrt`` / ``Math.Sin`` — the
    baseline its "CPU+GPU 3x as fast" comment (Kamera.cs:266) is measured
    against.  The loop is native and scalar (``cek.wave_reference_scalar``,
    csrc/refloops.cpp), as the .NET JIT runs it."""

    def __init__(self, base: np.ndarray, normals: np.ndarray):
        if base.dtype != VERTEX or normals.dtype != VERTEX or len(base) != len(normals):
            raise ValueError("base and normals must be equal-length VERTEX arrays")
        from .._native import cek

        self._cek = cek
        self.n = len(base)
        self.base = np.ascontiguousarray(base)
        self.normals = np.ascontiguousarray(normals)
        self.vertices = self.base.copy()
        self.t = 0.0
        self.ctr = 0.0

    def update(self) -> np.ndarray:
        if self.ctr < 0.3:
            self.ctr += 0.001
        self.t += 0.001
        self._cek.wave_reference_scalar(self.base.ctypes.data, self.normals.ctypes.data, self.vertices.ctypes.data,
                                        self.n, float(self.ctr), float(self.t))
        return self.vertices

    def reference(self) -> np.ndarray:
        return wave_reference(self.base, self.normals, np.float32(self.ctr), np.float32(self.t),
                              self.base["x"][0], self.base["y"][0])
