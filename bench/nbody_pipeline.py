"""BASELINE config 4: N-body (1M bodies) as a 3-stage device-to-device
pipeline, double-buffered, stage transitions over xGMI (peer copies on the
native copy engine, no host bounce).

  stage 1: all-pairs forces (LDS-tiled, rsqrt, packed pairs) — O(n²), the
           force stage is range-split over its GPUs by the load balancer
  stage 2: leapfrog kick-drift                                 — O(n)
  stage 3: kinetic-energy diagnostic (per-group sums) + state pass-through

Time stepping.  Step t+1 of one system needs step t's kick output, so a
single system cannot keep three stages busy: its next input exists only once
it has left the pipeline (latency L = 2·stages pushes).  The pipeline
therefore carries M = L + 1 systems of n bodies in rotation: push k feeds
system k mod M its current state, the state that leaves the pipeline at
push k + L is written back, and that system is fed again at push k + M.
Every system is genuinely time-stepped (state carried from step to step);
every push advances one system by one step through all three stages.  The
first stepped system is checked against a float64 host step on sampled
bodies.

Placement (BASELINE config 4: 4 GPUs).  ``shared`` (default): every stage
spans every GPU — the stages share devices, as the reference allows
(ClPipeline.cs:1728) — so the O(n²) force stage is range-split over all of
them and the O(n) kick and energy stages run beside it on their own
streams; no GPU idles for a push.  ``split``: distinct GPUs per stage
(force on all but two, kick and energy on one each: 2 + 1 + 1 on four), the
round-3 placement whose last two GPUs sat idle 99 % of a push.
``--logical 4`` rehearses the four-GPU placement on one GPU (four logical
devices of GPU 0).  ``device_busy_fraction``: per device, the union of its
kernel spans (every stage) over the steady pushes' wall time.  Stage times
are device times from hipEvent timelines; the stage-transition copies are
timed by hipEvents on the copy engine's streams, and both are put on one
host-anchored clock, so ``copy_overlap`` measures how much of the transfer
time ran while the force stage was computing (1.0 = fully hidden).  Kernels
are user kernel strings JIT-compiled by hiprtc.
"""
import argparse
import time

import numpy as np

from common import FP32_PEAK_TFLOPS, emit, sync

import cekirdekler_amd as ck
from cekirdekler_amd._native import cek
from cekirdekler_amd.parallel.pipeline import ClPipelineStage, _intersection

FORCE = r"""
// 2 bodies per work item as one packed f32x2 pair (v_pk_* issue: see
// kernels/nbody.hip), written as a user kernel string and JIT-compiled by
// hiprtc.  j-split: the work-group's 256 threads are two groups of 128 that
// hold the same 256 bodies (work-group g owns bodies [256 g, 256 g + 256),
// so a device's range of whole work-groups owns one contiguous body range)
// and take the two halves of every 512-body LDS load; the halves' partial
// accelerations are added through LDS at the end.  Twice the waves of a
// 2-bodies-per-item kernel for the same body share: with a quarter of the
// bodies per GPU (the force stage on four GPUs) that is 51.0 % of the FP32
// peak against 48.9 % (tools/nbody_force_variants.py, profiles/round4_session2.md).
// The next LDS load is held in registers while the current one is consumed.
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void force(const float4* pos, const float4* vel, const float* prm,
                                             float4* pos_o, float4* vel_o, float4* acc_o) {
  __shared__ float4 tile[512];
  const int n = (int)prm[2];
  const f2 e2 = {prm[0], prm[0]};
  const int l = threadIdx.x, grp = l >> 7, m = l & 127;
  const long long i0 = (get_global_id(0) / 256) * 256 + m;  // bodies i0 and i0 + 128
  const float4 b0 = pos[i0], b1 = pos[i0 + 128];
  const f2 px = {b0.x, b1.x}, py = {b0.y, b1.y}, pz = {b0.z, b1.z};
  f2 ax = {0.f, 0.f}, ay = ax, az = ax;
  float4 nx0 = pos[l], nx1 = pos[256 + l];
  for (int j0 = 0; j0 < n; j0 += 512) {
    __syncthreads();
    tile[l] = nx0;
    tile[256 + l] = nx1;
    __syncthreads();
    if (j0 + 512 < n) {
      nx0 = pos[j0 + 512 + l];
      nx1 = pos[j0 + 768 + l];
    }
    const float4* tg = tile + grp * 256;
#pragma unroll 8
    for (int j = 0; j < 256; ++j) {
      const float4 q = tg[j];
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
  __syncthreads();
  float* red = (float*)tile;
  if (grp == 1) {
    float* r = red + m * 6;
    r[0] = ax.x; r[1] = ax.y; r[2] = ay.x; r[3] = ay.y; r[4] = az.x; r[5] = az.y;
  }
  __syncthreads();
  if (grp == 0) {
    const float* r = red + m * 6;
    ax += f2{r[0], r[1]}; ay += f2{r[2], r[3]}; az += f2{r[4], r[5]};
    acc_o[i0] = make_float4(ax.x, ay.x, az.x, 0.f);
    acc_o[i0 + 128] = make_float4(ax.y, ay.y, az.y, 0.f);
    pos_o[i0] = b0; pos_o[i0 + 128] = b1;
    vel_o[i0] = vel[i0]; vel_o[i0 + 128] = vel[i0 + 128];
  }
}
"""
KICK = r"""
__global__ void kick(const float4* pos, const float4* vel, const float4* acc, const float* prm,
                     float4* pos_o, float4* vel_o) {
  long long i = get_global_id(0);
  float dt = prm[3];
  float4 p = pos[i], v = vel[i], a = acc[i];
  v.x += a.x * dt; v.y += a.y * dt; v.z += a.z * dt;
  p.x += v.x * dt; p.y += v.y * dt; p.z += v.z * dt;
  pos_o[i] = p; vel_o[i] = v;
}
"""
ENERGY = r"""
__global__ __launch_bounds__(256) void energy(const float4* pos, const float4* vel, float4* pos_o, float4* vel_o,
                                              float* e_o) {
  __shared__ float s[256];
  long long i = get_global_id(0);
  float4 p = pos[i], v = vel[i];
  pos_o[i] = p; vel_o[i] = v;
  s[threadIdx.x] = 0.5f * p.w * (v.x * v.x + v.y * v.y + v.z * v.z);
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) { if (threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w]; __syncthreads(); }
  if (threadIdx.x == 0) e_o[get_global_id(0) / 256] = s[0];
}
"""


def host_step(pos, vel, prm, idx):
    """float64 leapfrog kick-drift of bodies ``idx`` (forces from all bodies)."""
    eps2, dt = float(prm[0]), float(prm[3])
    p = pos.astype(np.float64)
    out_p, out_v = [], []
    for i in idx:
        d = p[:, :3] - p[i, :3]
        r2 = (d * d).sum(1) + eps2
        inv = 1.0 / np.sqrt(r2)
        acc = (d * (p[:, 3] * inv ** 3)[:, None]).sum(0)
        v = vel[i, :3].astype(np.float64) + acc * dt
        out_v.append(v)
        out_p.append(p[i, :3] + v * dt)
    return np.array(out_p), np.array(out_v)


ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1 << 20)
ap.add_argument("--pushes", type=int, default=14)
ap.add_argument("--gpus", type=int, default=0, help="0 = all visible")
ap.add_argument("--logical", type=int, default=0, help="rehearsal: act as if GPU 0 were this many GPUs")
ap.add_argument("--placement", choices=("shared", "split"), default="shared")
ap.add_argument("--cu-partition", type=int, choices=(0, 1), default=1,
                help="with --logical: the logical devices are disjoint CU partitions of GPU 0 (default) "
                     "or share all of its CUs")
a = ap.parse_args()
n = a.n
g = ck.ClPlatforms.all().gpus()
if a.logical > 1 and a.cu_partition:
    # four logical devices that each own a quarter of the
    # CUs (every XCD represented): the 4-GPU placement with each "GPU" a
    # disjoint CU set, so device busy fractions mean what they would on 4 GPUs
    g = g[0:1].cu_partitions(a.logical)
elif a.logical > 1:
    g0 = g[0]
    for _ in range(a.logical - 1):
        g0 = g0 + g[0]
    g = g0
ng = len(g) if a.gpus <= 0 else min(a.gpus, len(g))
if a.placement == "shared":
    # every stage on every GPU: device index k of each stage is GPU k
    devs = [g[0:ng]] * 3
    dev_of = [list(range(ng))] * 3
elif ng >= 3:
    # distinct GPUs per stage: the O(n²) force stage gets every GPU but the
    # last two (range-split by the load balancer); kick-drift and the energy
    # diagnostic get one each
    devs = [g[0:ng - 2], g[ng - 2], g[ng - 1]]
    dev_of = [list(range(ng - 2)), [ng - 2], [ng - 1]]
else:
    devs = [g[i % ng] for i in range(3)]
    dev_of = [[i % ng] for i in range(3)]

f4 = lambda: np.zeros(4 * n, np.float32)  # noqa: E731
prm = np.array([1e-4, 1.0, float(n), 1e-3], np.float32)
s1, s2, s3 = ClPipelineStage(), ClPipelineStage(), ClPipelineStage()
s1.add_devices(devs[0]); s1.add_kernels(FORCE, "force", [n], [256])
s1.add_input_buffers(f4(), f4()); s1.add_hidden_buffers(prm.copy()); s1.add_output_buffers(f4(), f4(), f4())
s2.add_devices(devs[1]); s2.add_kernels(KICK, "kick", [n], [256])
s2.add_input_buffers(f4(), f4(), f4()); s2.add_hidden_buffers(prm.copy()); s2.add_output_buffers(f4(), f4())
s3.add_devices(devs[2]); s3.add_kernels(ENERGY, "energy", [n], [256])
s3.add_input_buffers(f4(), f4()); s3.add_output_buffers(f4(), f4(), np.zeros(n // 256, np.float32))
# slice ownership in multi-device stages: a force, kick or energy work item
# owns one body (4 floats) of each output (a force work-group of 256 items
# holds 256 bodies), an energy work-group one partial sum
for arr in s1.outputs + s2.outputs + s3.outputs[:2]:
    arr.elements_per_work_item = 4
s3.outputs[2].elements_per_group = 1
s1.prepend_to_stage(s2)
s2.prepend_to_stage(s3)
pipe = s1.make_pipeline()
pipe.record_timeline = True
S = 3
L = 2 * S                 # a push's data leaves the pipeline L pushes later
M = L + 1                 # systems in rotation
rng = np.random.default_rng(0)
states = []
for _ in range(M):
    pos = np.zeros((n, 4), np.float32)
    vel = np.zeros((n, 4), np.float32)
    pos[:, :3] = rng.standard_normal((n, 3))
    pos[:, 3] = 1.0 / n
    vel[:, :3] = 0.01 * rng.standard_normal((n, 3))
    states.append([pos, vel])
steps = [0] * M
first_in = [states[0][0].copy(), states[0][1].copy()]
res_pos, res_vel = np.zeros((n, 4), np.float32), np.zeros((n, 4), np.float32)
energy = np.zeros(n // 256, np.float32)
kinetic = {}
times, ready_at, check = [], None, None
windows = []  # (begin, end) of every push on the runtime clock
for k in range(a.pushes):
    j = k % M
    sync()
    t = time.perf_counter()
    w0 = cek.now_ms()
    ready = pipe.push_data([states[j][0].reshape(-1), states[j][1].reshape(-1)],
                           [res_pos.reshape(-1), res_vel.reshape(-1), energy])
    sync()
    windows.append((w0, cek.now_ms()))
    times.append((time.perf_counter() - t) * 1e3)
    if ready:
        if ready_at is None:
            ready_at = k
        done = (k - L) % M   # the system fed L pushes ago
        states[done][0][:] = res_pos
        states[done][1][:] = res_vel
        steps[done] += 1
        kinetic.setdefault(done, []).append(float(energy.sum()))
        if done == 0 and steps[0] == 1:
            idx = np.random.default_rng(1).choice(n, 8, replace=False)
            hp, hv = host_step(first_in[0], first_in[1], prm, idx)
            err_p = np.abs(res_pos[idx, :3] - hp).max() / np.abs(hp).max()
            err_v = np.abs(res_vel[idx, :3] - hv).max() / np.abs(hv).max()
            check = float(max(err_p, err_v))
steady = times[L:] if len(times) > L + 1 else times[2:]
ms = float(np.median(steady))


tl = pipe.timeline()


def stage_device_ms(i):
    """Median per-push kernel time of stage i: each push is one compute per
    device; a push costs the stage its slowest device's span."""
    per_dev = {}
    for st, d, b, e in tl["kernels"]:
        if st == i:
            per_dev.setdefault(d, []).append(e - b)
    rows = [max(v[k] for v in per_dev.values()) for k in range(min(len(v) for v in per_dev.values()))]
    rows = rows[-len(steady):] if len(rows) > len(steady) else rows
    return float(np.median(rows))


stage_ms = [stage_device_ms(i) for i in range(3)]


def device_busy_fraction():
    """Per device of the placement (logical devices count separately): the
    union of its kernel spans, every stage, inside the steady pushes'
    windows, over those windows' total length."""
    skip = L if len(windows) > L + 1 else 2
    wins = [(b - tl["t0"], e - tl["t0"]) for b, e in windows[skip:]]
    total = sum(e - b for b, e in wins)
    spans = {}
    for st, d, b, e in tl["kernels"]:
        spans.setdefault(dev_of[st][d], []).append((b, e))
    out = []
    for dev in range(ng):
        iv = spans.get(dev, [])
        union = []
        for b, e in sorted(iv):
            if union and b <= union[-1][1]:
                union[-1][1] = max(union[-1][1], e)
            else:
                union.append([b, e])
        busy = sum(_intersection(wb, we, [tuple(u) for u in union]) for wb, we in wins)
        out.append(round(busy / total, 4) if total > 0 else 0.0)
    return out


busy = device_busy_fraction()
ov_force = pipe.copy_overlap(tl, stage=0)
ov_any = pipe.copy_overlap(tl)
xfer = pipe.transfer_stats()
emit({"config": "nbody_pipeline_3stage", "n": n, "systems_in_flight": M, "gpus_used": ng,
      "placement_mode": a.placement, "stage_gpus": [len(d) if hasattr(d, "__len__") else 1 for d in devs],
      "push_ms_median": ms, "device_busy_fraction": busy, "min_device_busy_fraction": min(busy),
      "stage_device_ms": stage_ms, "ready_after_pushes": ready_at,
      "interactions_per_s": n * n / (ms * 1e-3), "tflops_20flop": 20 * n * n / (ms * 1e-3) / 1e12,
      # per PHYSICAL GPU of the force stage (logical devices of one GPU share it)
      "force_stage_pct_fp32_peak": 100 * 20 * n * n / (stage_ms[0] * 1e-3) / 1e12 / FP32_PEAK_TFLOPS
      / len({devs[0].device(k).info.ordinal for k in range(len(devs[0]))}),
      "overlap_efficiency": max(stage_ms) / ms, "serial_over_push": sum(stage_ms) / ms,
      "steps_per_system": steps, "step_check_max_rel_err": check,
      "logical_rehearsal": a.logical > 1, "cu_partitioned": bool(a.logical > 1 and a.cu_partition),
      "placement": [[d.device(k).name + f"#{d.device(k).info.ordinal}" + (
          f"/cu{d.device(k).cu_partition[0]}of{d.device(k).cu_partition[1]}" if d.device(k).cu_partition else "")
                                                           for k in range(len(d))] for d in devs],
      "copy_ms_per_push": ov_any["copy_ms"] / a.pushes,
      "copy_overlap": {"with_force_stage": round(ov_force["fraction"], 4),
                       "with_any_stage": round(ov_any["fraction"], 4),
                       "copy_ms_total": round(ov_any["copy_ms"], 3), "copies": len(tl["copies"])},
      "transfer_bytes": xfer, "kinetic_energy_system0": kinetic.get(0, [])})
pipe.dispose()
if check is None or not check < 1e-3:
    raise SystemExit(f"nbody step check failed: {check}")
