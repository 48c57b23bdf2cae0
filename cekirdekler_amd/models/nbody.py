"""All-pairs N-body simulation on the AOT CDNA4 kernels.

The body range is split across devices by the load balancer; one compute()
runs the force kernel and the kick-drift kernel on the same balanced range.  Every device needs every position for the
force pass, so after each step the position slices are made coherent again:

* ``resident=True`` (MI355X-native): positions stay in device memory and each
  device's updated slice is copied into the other devices' replicas by the
  keep-resident gather flag (``ClArray.gather_resident``: event-ordered
  GPU↔GPU peer copies over xGMI inside the compute, no host sync);
* ``resident=False`` (reference semantics, Tester.cs:7759-7765): slices go
  device→host and the whole array host→device on the next step.
"""
from __future__ import annotations

import numpy as np

from ..arrays import ClArray
from ..cruncher import ClNumberCruncher
from ..ops.library import library

FLOP_PER_INTERACTION = 20
L = 256


def nbody_accel_reference(pos: np.ndarray, eps2: float, g: float = 1.0, chunk: int = 1024) -> np.ndarray:
    """float64 all-pairs reference: a_i = G Σ_j m_j (x_j − x_i) / (|x_j − x_i|² + ε²)^{3/2}."""
    p = pos.reshape(-1, 4).astype(np.float64)
    out = np.zeros((len(p), 3))
    for s in range(0, len(p), chunk):
        d = p[None, :, :3] - p[s:s + chunk, None, :3]
        r2 = (d * d).sum(-1) + eps2
        inv3 = r2 ** -1.5
        out[s:s + chunk] = g * (d * (p[None, :, 3] * inv3)[..., None]).sum(1)
    return out


class NBodySimulation:
    def __init__(self, n: int, devices=None, cruncher: ClNumberCruncher | None = None, eps: float = 0.01,
                 dt: float = 1e-3, g: float = 1.0, seed: int = 0, resident: bool = True,
                 bodies_per_item: int | None = None):
        # 4 bodies per work item once the grid still has >= 4 workgroups per
        # CU (n >= 1M on 256 CUs); 2 below that, for occupancy
        b = bodies_per_item or (4 if n >= 4 * L * 1024 else 2)
        if b not in (2, 4):
            raise ValueError("bodies_per_item must be 2 or 4")
        if n % (b * L):
            raise ValueError(f"n must be a multiple of {b * L}")
        self.n = n
        self.bpw = b
        self.k_force, self.k_integrate = f"cek_nbody_f32_b{b}", f"cek_nbody_integrate_f32_b{b}"
        self.k_energy = f"cek_nbody_energy_f32_b{b}"
        self.resident = resident
        self.cr = cruncher or ClNumberCruncher(devices, "", prebuilt=library("nbody"))
        rng = np.random.default_rng(seed)
        pos = np.empty((n, 4), np.float32)
        pos[:, :3] = rng.standard_normal((n, 3)).astype(np.float32)
        pos[:, 3] = 1.0 / n
        self.pos = ClArray(pos.reshape(-1))
        self.vel = ClArray(np.zeros(4 * n, np.float32))
        self.acc = ClArray(np.zeros(4 * n, np.float32))
        self.params = ClArray(np.array([eps * eps, g, float(n), dt], np.float32))
        self.params.write = False
        self.steps = 0

    @property
    def interactions_per_step(self) -> float:
        return float(self.n) * float(self.n)

    @property
    def flops_per_step(self) -> float:
        return FLOP_PER_INTERACTION * self.interactions_per_step

    def _flags(self) -> None:
        first = self.steps == 0
        for a in (self.pos, self.vel, self.acc):
            a.elements_per_work_item = 4 * self.bpw  # bpw bodies × float4 per work item
            a.partial_read = False
        # positions: every device reads all of them
        self.pos.read = first or not self.resident
        self.pos.write = not self.resident
        self.pos.gather_resident = self.resident
        self.vel.partial_read = not self.resident or first
        self.vel.read = False
        self.vel.write = not self.resident
        self.acc.read = False
        self.acc.write = False
        self.params.read = first or not self.resident

    def forces(self, compute_id: int = 3) -> None:
        """Accelerations only (no integration)."""
        self._flags()
        self.pos.write = False
        self.pos.gather_resident = False
        self.acc.write = True
        self.pos.next_param(self.vel, self.acc, self.params).compute(self.cr, compute_id, self.k_force,
                                                                    self.n // self.bpw, L)

    def step(self, compute_id: int = 1) -> None:
        """Forces + kick-drift for every body, range-partitioned; then the
        position slices are made coherent on every device."""
        self._flags()
        self.pos.next_param(self.vel, self.acc, self.params).compute(
            self.cr, compute_id, f"{self.k_force} {self.k_integrate}", self.n // self.bpw, L)
        self.steps += 1

    def download(self) -> None:
        """Bring device-resident state to the host (device 0 holds every
        slice of pos after the gather; vel/acc slices per device)."""
        if not self.resident:
            return  # host arrays already hold every slice
        c = self.cr.cores
        self.cr.download(self.pos, 0)
        for name in ("vel", "acc"):
            arr = getattr(self, name)
            if c.num_devices == 1:
                self.cr.download(arr, 0)
                continue
            cid = 1
            refs, rng = self.cr.references(cid), self.cr.ranges(cid)
            e = 4 * self.bpw
            full = np.empty_like(arr.array)
            keep = arr.array.copy()
            for d in range(c.num_devices):
                self.cr.download(arr, d)
                g = c.global_base + d
                full[refs[g] * e:(refs[g] + rng[g]) * e] = arr.array[refs[g] * e:(refs[g] + rng[g]) * e]
            keep[:] = full
            arr.array[:] = keep
