#!/bin/bash
# Builds the GEMM main-loop probe (shipped kernels / L2-resident operands).
cd "$(dirname "$0")"
hipcc --offload-arch=gfx950 -O3 -std=c++17 gemm_loop.hip -o gemm_loop &&
hipcc --offload-arch=gfx950 -O3 -std=c++17 -DCEK_PROBE_L2 gemm_loop.hip -o gemm_loop_l2 &&
hipcc --offload-arch=gfx950 -O3 -std=c++17 -DCEK_PROBE_TS gemm_loop.hip -o gemm_loop_ts
