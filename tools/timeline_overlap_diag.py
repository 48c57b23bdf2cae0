"""GPU diagnostic: DevicePipeline two-stage overlap per measurement window,
first instance in a fresh process vs a second one (the stage kernels'
hipEvent spans, relative ms)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cekirdekler_amd as ck  # noqa: E402
from cekirdekler_amd.parallel.pipeline import (DevicePipeline, DevicePipelineArray,  # noqa: E402
                                               DevicePipelineArrayType, DevicePipelineStage)

gpu = ck.ClPlatforms.all().gpus()
N = 1 << 14
body = "float v = x[i]; for (int j = 0; j < 200000; ++j) v = v * 0.9999f + 0.5f;"
src = ("__global__ void s0(const float* x, float* y) { long long i = get_global_id(0); " + body + " y[i] = v; }\n"
       "__global__ void s1(const float* x, float* y) { long long i = get_global_id(0); " + body + " y[i] = v; }")
out = {}
for inst in range(2):
    dp = DevicePipeline(gpu[0], src)
    arrs = [DevicePipelineArray(DevicePipelineArrayType.INPUT, np.ones(N, np.float32)) for _ in range(2)]
    outs = [DevicePipelineArray(DevicePipelineArrayType.OUTPUT, np.zeros(N, np.float32)) for _ in range(2)]
    for k in range(2):
        st = DevicePipelineStage(f"s{k}", N, 256)
        st.bind_array(arrs[k])
        st.bind_array(outs[k])
        dp.add_stage(st)
    for _ in range(18):
        dp.feed()
    wins = []
    for w in range(4):
        dp.record_timeline = True
        for _ in range(3):
            dp.feed()
        spans = dp._collect()
        wins.append({"overlap": round(dp.query_timeline_overlap_percentage(), 1),
                     "spans": [(s, round(b, 3), round(e, 3)) for s, b, e in spans]})
    out[f"instance{inst}"] = {"qconc": dp.cruncher.compute_queue_concurrency, "windows": wins}
    dp.dispose()
print(json.dumps(out), flush=True)
