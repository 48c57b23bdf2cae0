#!/bin/bash
# Round-4 probes on one GPU: host fan-out cost and pool throughput (both
# worker hand-off modes), PCIe duplex beside a CU-masked busy kernel, and
# the N-body force-kernel variants, register-direct fp32 GEMM tiles.  Each step has its own time limit; the
# first failing step ends the call.
set -o pipefail
out=${1:-gpurun_out/probes}
mkdir -p "$out"
timeout -k 10 240 python tools/scale_probe.py 1024,8192 256x256pbw,256x256pbh,256x256pbs,256x256pb,256x256pb:a 3 20 > "$out/scale_probe.json" 2> "$out/scale_probe.err" || exit $?
timeout -k 10 240 python tools/gemm_f32_probe.py 8192 256x256ir,256x256gt,256x256g8t,256x256g,256x256g8 3 5 > "$out/f32_probe.json" 2> "$out/f32_probe.err" || exit $?
for v in "4 sw" "4 sh" "0 ss" "1 ss" "2 ss"; do
  timeout -k 10 60 ./tools/microbench/gemm_loop 30 $v >> "$out/gemm_loop.json" 2>> "$out/gemm_loop.err" || exit $?
done
for v in "4 sw" "4 sh" "0 ss"; do
  timeout -k 10 60 ./tools/microbench/gemm_loop_ts 10 $v >> "$out/gemm_loop_ts.json" 2>> "$out/gemm_loop.err" || exit $?
done
CEK_POOL_SPIN_US=0 timeout -k 10 120 python tools/cpu_spin_probe.py "$out/cpu_spin0.json" > /dev/null 2>> "$out/cpu_spin.err" || exit $?
CEK_POOL_SPIN_US=50 timeout -k 10 120 python tools/cpu_spin_probe.py "$out/cpu_spin50.json" > /dev/null 2>> "$out/cpu_spin.err" || exit $?
CEK_SPIN_US=0 timeout -k 10 180 python tools/fanout_probe.py "$out/fanout_spin0.json" > "$out/fanout0.log" 2>&1 || exit $?
timeout -k 10 180 python tools/fanout_probe.py "$out/fanout_spin50.json" > "$out/fanout50.log" 2>&1 || exit $?
timeout -k 10 120 ./tools/microbench/pcie_cumask > "$out/pcie_cumask.json" 2> "$out/pcie_cumask.err" || exit $?
timeout -k 10 240 python tools/nbody_force_variants.py 1048576 1,0.5,0.25 "$out/nbody_variants.json" > "$out/nbody_variants.log" 2>&1 || exit $?
timeout -k 10 240 python bench/nbody_pipeline.py --gpus 4 --logical 4 --pushes 12 > "$out/nbody_shared.json" 2> "$out/nbody_shared.err" || exit $?
