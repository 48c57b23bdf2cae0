"""Selectable device-function prelude for kernel strings.

The reference declares ``ClBuiltInAuxilliaryFunctions`` with one stub
(``exampleFunction``) and marks it "not implemented (yet)"
(src/ClBuiltInAuxilliaryFunctions.cs:28-47).  Here it is a working prelude
builder: switch helpers on, then prepend ``str(aux)`` (or ``aux.wrap(src)``)
to a kernel string.  Every helper compiles for both targets — gfx950 via
hiprtc and the host CPU device via the host compiler (the CPU prelude runs
work-items of a group as fibers, so the LDS-based block helpers work there
too; the wave-level helpers fall back to the block path on the CPU).
"""
from __future__ import annotations

from typing import Dict, List

_FUNCS: Dict[str, str] = {
    # the reference stub, with its declared return type fixed (it returns a+b)
    "example_function": "__device__ inline int exampleFunction(int a, int b) { return a + b; }\n",
    "clamp01": "__device__ inline float cek_clamp01(float x) { return x < 0.f ? 0.f : (x > 1.f ? 1.f : x); }\n",
    "lerp": "__device__ inline float cek_lerp(float a, float b, float t) { return a + t * (b - a); }\n",
    "bf16": r"""
__device__ inline float cek_bf16_to_f32(unsigned short h) {
  union { unsigned int u; float f; } c; c.u = ((unsigned int)h) << 16; return c.f; }
__device__ inline unsigned short cek_f32_to_bf16(float f) {   // round to nearest even
  union { unsigned int u; float f; } c; c.f = f;
  unsigned int r = 0x7fffu + ((c.u >> 16) & 1u);
  return (unsigned short)((c.u + r) >> 16); }
""",
    # 64-wide wavefront reduction (CDNA4 wave64; DPP/swizzle via __shfl_xor)
    "wave_sum": r"""
#ifdef CEK_GPU
__device__ inline float cek_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v; }
#endif
""",
    # workgroup reduction through LDS; every work item gets the sum.
    # scratch must hold blockDim.x floats (declare it __shared__ in the kernel)
    "block_sum": r"""
__device__ inline float cek_block_sum(float v, float* scratch) {
  const int t = (int)get_local_id(0), n = (int)get_local_size(0);
  scratch[t] = v;
  __syncthreads();
  for (int s = n / 2; s > 0; s >>= 1) {
    if (t < s) scratch[t] += scratch[t + s];
    __syncthreads();
  }
  const float r = scratch[0];
  __syncthreads();
  return r; }
""",
}


class ClBuiltInAuxilliaryFunctions:
    """Flags select helpers; ``str()`` yields the prelude text."""

    NAMES: List[str] = list(_FUNCS)
    ALIASES = {"exampleFunction": "example_function"}   # reference spelling

    def __init__(self, **enabled: bool):
        self._on = {k: False for k in _FUNCS}
        for k, v in enabled.items():
            setattr(self, k, v)

    def __getattr__(self, name):
        name = self.ALIASES.get(name, name)
        on = self.__dict__.get("_on")
        if on is not None and name in on:
            return on[name]
        raise AttributeError(name)

    def __setattr__(self, name, value):
        name = self.ALIASES.get(name, name)
        if name != "_on" and name in _FUNCS:
            self._on[name] = bool(value)
        elif name == "_on":
            object.__setattr__(self, name, value)
        else:
            raise AttributeError(f"unknown auxiliary function {name!r}; known: {', '.join(_FUNCS)}")

    def enable_all(self) -> "ClBuiltInAuxilliaryFunctions":
        for k in self._on:
            self._on[k] = True
        return self

    def __str__(self) -> str:
        return "".join(_FUNCS[k] for k, v in self._on.items() if v)

    def wrap(self, kernel_source: str) -> str:
        return str(self) + "\n" + kernel_source
