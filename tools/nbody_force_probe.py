"""GPU probe: the N-body pipeline's force kernel (bench/nbody_pipeline.py,
JIT-compiled user string) on one GPU at a fraction of the bodies, i.e. the
share one GPU computes when the force stage spans 1, 2 or 4 GPUs.

    python tools/nbody_force_probe.py [n] [fractions]
"""
import json
import os
import re
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402

src = open(os.path.join(ROOT, "bench", "nbody_pipeline.py")).read()
kernels = {name: re.search(name + r' = r"""(.*?)"""', src, re.S).group(1) for name in ("FORCE",)}
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
fracs = [float(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,0.5,0.25").split(",")]
g0 = ck.ClPlatforms.all().gpus()[0]
FORCE2 = r"""
// 2 bodies per work item (one packed pair): twice the work-groups of force
__global__ __launch_bounds__(256) void force2(const float4* pos, const float4* vel, const float* prm,
                                              float4* pos_o, float4* vel_o, float4* acc_o) {
  __shared__ float4 tile[256];
  const int n = (int)prm[2];
  const f2 e2 = {prm[0], prm[0]};
  const long long w = get_global_id(0);
  const long long i0 = (w / 256) * 512 + (w % 256);
  float4 b0 = pos[i0], b1 = pos[i0 + 256];
  f2 px = {b0.x, b1.x}, py = {b0.y, b1.y}, pz = {b0.z, b1.z};
  f2 ax = {0.f, 0.f}, ay = ax, az = ax;
  for (int j0 = 0; j0 < n; j0 += 256) {
    __syncthreads();
    tile[threadIdx.x] = pos[j0 + threadIdx.x];
    __syncthreads();
#pragma unroll 8
    for (int j = 0; j < 256; ++j) {
      const float4 q = tile[j];
      const f2 qx = {q.x, q.x}, qy = {q.y, q.y}, qz = {q.z, q.z}, qm = {q.w, q.w};
      const f2 dx = qx - px, dy = qy - py, dz = qz - pz;
      const f2 r2 = __builtin_elementwise_fma(dx, dx, __builtin_elementwise_fma(dy, dy, __builtin_elementwise_fma(dz, dz, e2)));
      const f2 inv = {__builtin_amdgcn_rsqf(r2.x), __builtin_amdgcn_rsqf(r2.y)};
      const f2 sc = (qm * inv) * (inv * inv);
      ax = __builtin_elementwise_fma(dx, sc, ax);
      ay = __builtin_elementwise_fma(dy, sc, ay);
      az = __builtin_elementwise_fma(dz, sc, az);
    }
  }
  acc_o[i0] = make_float4(ax.x, ay.x, az.x, 0.f);
  acc_o[i0 + 256] = make_float4(ax.y, ay.y, az.y, 0.f);
  pos_o[i0] = pos[i0]; pos_o[i0 + 256] = pos[i0 + 256];
  vel_o[i0] = vel[i0]; vel_o[i0 + 256] = vel[i0 + 256];
}
"""
extra = sys.argv[3] if len(sys.argv) > 3 else FORCE2
cr = ck.ClNumberCruncher(g0, kernels["FORCE"] + extra)
rng = np.random.default_rng(0)
pos = np.zeros((n, 4), np.float32)
pos[:, :3] = rng.standard_normal((n, 3))
pos[:, 3] = 1.0 / n
vel = np.zeros((n, 4), np.float32)
prm = np.array([1e-4, 1.0, float(n), 1e-3], np.float32)
arrs = [ck.ClArray(pos.reshape(-1)), ck.ClArray(vel.reshape(-1)), ck.ClArray(prm)] + [
    ck.ClArray(np.zeros(4 * n, np.float32)) for _ in range(3)]
for a in arrs[:3]:
    a.write = False
for a in arrs[3:]:
    a.read = False
    a.write = False
res = {}
names = [k for k in ("force", "force2") if re.search(r"void " + k + r"\(", kernels["FORCE"] + extra)]
for kname in names:
    bodies_per_item = 4 if kname == "force" else 2
    for f in fracs:
        g = int(n // bodies_per_item * f) // 256 * 256
        call = lambda: arrs[0].next_param(*arrs[1:]).compute(cr, 1 + len(res), kname, g, 256)  # noqa: E731
        call()
        torch.cuda.synchronize()
        t = time.perf_counter()
        reps = 3
        for _ in range(reps):
            call()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3 / reps
        inter = g * bodies_per_item * n
        res[f"{kname}/{f}"] = {"work_groups": g // 256, "ms": round(ms, 2),
                              "tflops_20": round(20 * inter / ms / 1e9, 1),
                              "pct_fp32_peak": round(100 * 20 * inter / ms / 1e9 / 157.3, 1)}
print(json.dumps(res, indent=1))
cr.dispose()
