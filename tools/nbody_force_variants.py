"""GPU probe: variants of the N-body pipeline's JIT force kernel (user
kernel strings, hiprtc) on one GPU at the body share one GPU computes when
the force stage spans 1, 2 or 4 GPUs.  Same signature and body mapping as
bench/nbody_pipeline.py's FORCE (work-group g owns 256·B bodies).

    python tools/nbody_force_variants.py [n] [fractions] [out.json]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402

HEAD = "typedef float f2 __attribute__((ext_vector_type(2)));\n"


def variant(name, B, prefetch, tile, unroll):
    """B bodies per work item (B/2 packed pairs); `tile` bodies per LDS tile
    (256 or 512); `prefetch`: the next tile is loaded into registers while
    the current one is consumed."""
    NP = B // 2
    loads = tile // 256
    s = [f"__global__ __launch_bounds__(256) void {name}(const float4* pos, const float4* vel, const float* prm,",
         "    float4* pos_o, float4* vel_o, float4* acc_o) {",
         f"  __shared__ float4 t[{tile}];",
         "  const int n = (int)prm[2];",
         "  const f2 e2 = {prm[0], prm[0]};",
         "  const long long w = get_global_id(0);",
         f"  const long long i0 = (w / 256) * {256 * B} + (w % 256);",
         f"  f2 px[{NP}], py[{NP}], pz[{NP}], ax[{NP}], ay[{NP}], az[{NP}];",
         f"  for (int p = 0; p < {NP}; ++p) {{",
         "    const float4 b0 = pos[i0 + (2 * p) * 256], b1 = pos[i0 + (2 * p + 1) * 256];",
         "    px[p] = f2{b0.x, b1.x}; py[p] = f2{b0.y, b1.y}; pz[p] = f2{b0.z, b1.z};",
         "    ax[p] = ay[p] = az[p] = f2{0.f, 0.f};",
         "  }",
         "  const int l = threadIdx.x;"]
    if prefetch:
        s += [f"  float4 nx[{loads}];", f"  for (int k = 0; k < {loads}; ++k) nx[k] = pos[k * 256 + l];"]
    s += [f"  for (int j0 = 0; j0 < n; j0 += {tile}) {{", "    __syncthreads();"]
    if prefetch:
        s += [f"    for (int k = 0; k < {loads}; ++k) t[k * 256 + l] = nx[k];", "    __syncthreads();",
              f"    if (j0 + {tile} < n) for (int k = 0; k < {loads}; ++k) nx[k] = pos[j0 + {tile} + k * 256 + l];"]
    else:
        s += [f"    for (int k = 0; k < {loads}; ++k) t[k * 256 + l] = pos[j0 + k * 256 + l];", "    __syncthreads();"]
    s += [f"#pragma unroll {unroll}",
          f"    for (int j = 0; j < {tile}; ++j) {{",
          "      const float4 q = t[j];",
          "      const f2 qx = {q.x, q.x}, qy = {q.y, q.y}, qz = {q.z, q.z}, qm = {q.w, q.w};",
          "#pragma unroll",
          f"      for (int p = 0; p < {NP}; ++p) {{",
          "        const f2 dx = qx - px[p], dy = qy - py[p], dz = qz - pz[p];",
          "        const f2 r2 = __builtin_elementwise_fma(dx, dx, __builtin_elementwise_fma(dy, dy, __builtin_elementwise_fma(dz, dz, e2)));",
          "        const f2 inv = {__builtin_amdgcn_rsqf(r2.x), __builtin_amdgcn_rsqf(r2.y)};",
          "        const f2 sc = (qm * inv) * (inv * inv);",
          "        ax[p] = __builtin_elementwise_fma(dx, sc, ax[p]);",
          "        ay[p] = __builtin_elementwise_fma(dy, sc, ay[p]);",
          "        az[p] = __builtin_elementwise_fma(dz, sc, az[p]);",
          "      }", "    }", "  }",
          f"  for (int p = 0; p < {NP}; ++p) {{",
          "    const long long a = i0 + (2 * p) * 256, b = a + 256;",
          "    acc_o[a] = make_float4(ax[p].x, ay[p].x, az[p].x, 0.f);",
          "    acc_o[b] = make_float4(ax[p].y, ay[p].y, az[p].y, 0.f);",
          "    pos_o[a] = pos[a]; pos_o[b] = pos[b]; vel_o[a] = vel[a]; vel_o[b] = vel[b];",
          "  }", "}"]
    return "\n".join(s) + "\n"


def variant_js(name, B, S, mass_lds=False, unroll=8):
    """j-split: a work-group's 256 threads form S groups that take the same
    256·B/S bodies (B per thread, packed pairs) against S different 256-body
    tiles of each LDS load, and add their partial accelerations through LDS
    at the end: S times the waves for the same body share (more latency
    hiding when one GPU holds a quarter of the bodies).  A work item owns
    B/S bodies of each output.  ``mass_lds``: the masses also go to an LDS
    array of their own, so the body loop reads x, y, z (one 12-B read) and
    the masses of 4 bodies per 16-B read, and no VALU copy saves q.w from
    the register pair the z difference is written into."""
    NP, T = B // 2, 256 // S
    s = [f"__global__ __launch_bounds__(256) void {name}(const float4* pos, const float4* vel, const float* prm,",
         "    float4* pos_o, float4* vel_o, float4* acc_o) {",
         f"  __shared__ float4 t[{256 * S}];",
         f"  __shared__ float mt[{256 * S}];" if mass_lds else "",
         "  const int n = (int)prm[2];",
         "  const f2 e2 = {prm[0], prm[0]};",
         "  const int l = threadIdx.x;",
         f"  const int grp = l / {T}, m = l % {T};",
         f"  const long long i0 = (get_global_id(0) / 256) * {T * B} + m;  // pair p: bodies i0 + 2p·{T}, i0 + (2p+1)·{T}",
         f"  f2 px[{NP}], py[{NP}], pz[{NP}], ax[{NP}], ay[{NP}], az[{NP}];",
         f"  for (int p = 0; p < {NP}; ++p) {{",
         f"    const float4 b0 = pos[i0 + (2 * p) * {T}], b1 = pos[i0 + (2 * p + 1) * {T}];",
         "    px[p] = f2{b0.x, b1.x}; py[p] = f2{b0.y, b1.y}; pz[p] = f2{b0.z, b1.z};",
         "    ax[p] = ay[p] = az[p] = f2{0.f, 0.f};",
         "  }",
         f"  float4 nx[{S}];",
         f"  for (int k = 0; k < {S}; ++k) nx[k] = pos[k * 256 + l];",
         f"  for (int j0 = 0; j0 < n; j0 += {256 * S}) {{",
         "    __syncthreads();",
         f"    for (int k = 0; k < {S}; ++k) t[k * 256 + l] = nx[k];",
         f"    for (int k = 0; k < {S}; ++k) mt[k * 256 + l] = nx[k].w;" if mass_lds else "",
         "    __syncthreads();",
         f"    if (j0 + {256 * S} < n) for (int k = 0; k < {S}; ++k) nx[k] = pos[j0 + {256 * S} + k * 256 + l];",
         "    const float4* tg = t + grp * 256;",
         "    const float* mg = mt + grp * 256;" if mass_lds else "",
         f"#pragma unroll {unroll}",
         "    for (int j = 0; j < 256; ++j) {",
         "      const float4 q = tg[j];",
         "      const float qw = mg[j];" if mass_lds else "      const float qw = q.w;",
         "      const f2 qx = {q.x, q.x}, qy = {q.y, q.y}, qz = {q.z, q.z}, qm = {qw, qw};",
         "#pragma unroll",
         f"      for (int p = 0; p < {NP}; ++p) {{",
         "        const f2 dx = qx - px[p], dy = qy - py[p], dz = qz - pz[p];",
         "        const f2 r2 = __builtin_elementwise_fma(dx, dx, __builtin_elementwise_fma(dy, dy, __builtin_elementwise_fma(dz, dz, e2)));",
         "        const f2 inv = {__builtin_amdgcn_rsqf(r2.x), __builtin_amdgcn_rsqf(r2.y)};",
         "        const f2 sc = (qm * inv) * (inv * inv);",
         "        ax[p] = __builtin_elementwise_fma(dx, sc, ax[p]);",
         "        ay[p] = __builtin_elementwise_fma(dy, sc, ay[p]);",
         "        az[p] = __builtin_elementwise_fma(dz, sc, az[p]);",
         "      }", "    }", "  }",
         "  // groups 1..S-1 hand their partial sums to group 0 through LDS",
         "  __syncthreads();",
         "  float* red = (float*)t;",
         f"  if (grp > 0) for (int p = 0; p < {NP}; ++p) {{",
         f"    float* r = red + (((grp - 1) * {NP} + p) * {T} + m) * 6;",
         "    r[0] = ax[p].x; r[1] = ax[p].y; r[2] = ay[p].x; r[3] = ay[p].y; r[4] = az[p].x; r[5] = az[p].y;",
         "  }",
         "  __syncthreads();",
         "  if (grp == 0) {",
         f"    for (int g = 1; g < {S}; ++g) for (int p = 0; p < {NP}; ++p) {{",
         f"      const float* r = red + (((g - 1) * {NP} + p) * {T} + m) * 6;",
         "      ax[p] += f2{r[0], r[1]}; ay[p] += f2{r[2], r[3]}; az[p] += f2{r[4], r[5]};",
         "    }",
         f"    for (int p = 0; p < {NP}; ++p) {{",
         f"      const long long a = i0 + (2 * p) * {T}, b = a + {T};",
         "      acc_o[a] = make_float4(ax[p].x, ay[p].x, az[p].x, 0.f);",
         "      acc_o[b] = make_float4(ax[p].y, ay[p].y, az[p].y, 0.f);",
         "      pos_o[a] = pos[a]; pos_o[b] = pos[b]; vel_o[a] = vel[a]; vel_o[b] = vel[b];",
         "    }",
         "  }", "}"]
    return "\n".join(s) + "\n"


JS_VARIANTS = {"b2_js2": (2, 2), "b4_js2": (4, 2), "b2_js4": (2, 4),  # name: (B, S[, mass_lds])
               "b2_js2m": (2, 2, True), "b4_js2m": (4, 2, True), "b2_js4m": (2, 4, True),
               "b2_js2u4": (2, 2, False, 4), "b2_js2u16": (2, 2, False, 16), "b2_js2u32": (2, 2, False, 32)}

VARIANTS = {  # name: (B, prefetch, tile, unroll)
    "b2_plain": (2, False, 256, 8),
    "b2_pf": (2, True, 256, 8),
    "b2_pf512": (2, True, 512, 8),
    "b4_pf": (4, True, 256, 4),
    "b4_pf512": (4, True, 512, 4),
}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    fracs = [float(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,0.5,0.25").split(",")]
    src = HEAD + "".join(variant(k, *v) for k, v in VARIANTS.items()) + "".join(
        variant_js(k, *v) for k, v in JS_VARIANTS.items())
    # work items per body: B bodies per item, S items per body group for j-split
    per_item = {k: (v[0], 1) for k, v in VARIANTS.items()}
    per_item.update({k: (v[0], v[1]) for k, v in JS_VARIANTS.items()})
    if len(sys.argv) > 4:  # only the named variants
        keep = set(sys.argv[4].split(","))
        per_item = {k: v for k, v in per_item.items() if k in keep}
    g0 = ck.ClPlatforms.all().gpus()[0]
    cr = ck.ClNumberCruncher(g0, src)
    if cr.error_code():
        raise SystemExit(cr.error_message())
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
    cid = 1
    ref_acc = None
    for f in fracs:
        for name, (B, S) in per_item.items():
            g = int(n * S // B * f) // 256 * 256
            call = lambda: arrs[0].next_param(*arrs[1:]).compute(cr, cid, name, g, 256)  # noqa: E731
            call()
            torch.cuda.synchronize()
            best = 1e30
            for _ in range(3):
                t = time.perf_counter()
                call()
                torch.cuda.synchronize()
                best = min(best, (time.perf_counter() - t) * 1e3)
            bodies = g * B // S
            inter = bodies * n
            cr.download(arrs[5], 0)
            acc = arrs[5].array[: 4 * bodies].copy()
            if ref_acc is None or len(ref_acc) != len(acc):
                ref_acc = acc
            err = float(np.abs(acc - ref_acc).max() / max(np.abs(ref_acc).max(), 1e-30))
            res[f"{name}/{f}"] = {"work_groups": g // 256, "ms": round(best, 2),
                                  "pct_fp32_peak": round(100 * 20 * inter / best / 1e9 / 157.3, 1),
                                  "rel_diff_vs_first": err}
            print(name, f, res[f"{name}/{f}"], flush=True)
            cid += 1
    cr.dispose()
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
