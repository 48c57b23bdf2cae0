"""Device→device stage pipeline (reference ClPipeline): three stages, each
on its own device (round-robin over the GPUs, or the CPU device), double
buffered; results appear 2·stages pushes after their input."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np

import cekirdekler_amd as ck
from cekirdekler_amd.parallel.pipeline import ClPipelineStage

N = 1 << 16
K = {
    "add1": "__global__ void add1(const float* x, float* y) { long long i = get_global_id(0); y[i] = x[i] + 1.0f; }",
    "mul2": "__global__ void mul2(const float* x, float* y) { long long i = get_global_id(0); y[i] = x[i] * 2.0f; }",
    "sub3": "__global__ void sub3(const float* x, float* y) { long long i = get_global_id(0); y[i] = x[i] - 3.0f; }",
}
plats = ck.ClPlatforms.all()
pool = plats.gpus() if len(plats.gpus()) else plats.cpus(True)
stages = []
for s, name in enumerate(K):
    st = ClPipelineStage()
    st.add_devices(pool[s % len(pool)])
    st.add_kernels(K[name], name, [N], [256])
    st.add_input_buffers(np.zeros(N, np.float32))
    st.add_output_buffers(np.zeros(N, np.float32))
    stages.append(st)
stages[0].prepend_to_stage(stages[1])
stages[1].prepend_to_stage(stages[2])
pipe = stages[0].make_pipeline()
out = np.zeros(N, np.float32)
for p in range(10):
    if pipe.push_data([np.full(N, float(p), np.float32)], [out]):
        print(f"push {p}: result {out[0]:.1f}")   # ((p' + 1) * 2) - 3 for an earlier p'
pipe.dispose()
