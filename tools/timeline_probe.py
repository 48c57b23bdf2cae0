"""GPU probe: hipEvent timeline of a two-stage DevicePipeline in parallel
mode (one stream per stage), with the host time of each compute() call."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.parallel.pipeline import (DevicePipeline, DevicePipelineArray,  # noqa: E402
                                               DevicePipelineArrayType, DevicePipelineStage)

N = 1 << 14
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
body = f"float v = x[i]; for (int j = 0; j < {iters}; ++j) v = v * 0.9999f + 0.5f;"
src = "\n".join(f"__global__ void s{k}(const float* x, float* y) {{ long long i = get_global_id(0); {body} y[i] = v; }}"
                for k in range(2))
gpu = ck.ClPlatforms.all().gpus()
dp = DevicePipeline(gpu[0], src)
arrs = [DevicePipelineArray(DevicePipelineArrayType.INPUT, np.ones(N, np.float32)) for _ in range(2)]
outs = [DevicePipelineArray(DevicePipelineArrayType.OUTPUT, np.zeros(N, np.float32)) for _ in range(2)]
for k in range(2):
    st = DevicePipelineStage(f"s{k}", N, 256)
    st.bind_array(arrs[k])
    st.bind_array(outs[k])
    dp.add_stage(st)
for _ in range(18):  # both parities, all 16 compute streams used once
    dp.feed()
cr = dp.cruncher
cr.record_timeline = True
for f in range(3):
    t0 = time.perf_counter()
    cr.enqueue_mode = True
    cr.enqueue_mode_async_enable = True
    per = []
    for st in dp.stages:
        a = time.perf_counter()
        dp._args(st).compute(cr, 100 + st.index, st.kernel_names, st.global_range, st.local_range)
        per.append(1e3 * (time.perf_counter() - a))
    print("per-stage compute() host ms:", [round(x, 3) for x in per])
    t1 = time.perf_counter()
    dp._finish()
    t2 = time.perf_counter()
    print(f"feed {f}: enqueue {1e3 * (t1 - t0):.3f} ms, finish {1e3 * (t2 - t1):.3f} ms")
for t in cr.timeline():
    print(t)
dp.dispose()
