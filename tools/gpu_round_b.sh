#!/bin/bash
# Second GPU session of the round: the headline bench, its kernel trace, one
# counter pass over the fp32 GEMM tiles, then multi-rank rehearsals of the
# bench on the one GPU (ranks share GPU 0; the 8-GPU run is the driver's).
# Every step has its own time limit; a failing step ends the call.
set -o pipefail
out=${1:-gpurun_out/runb}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > "$out/bench.json" 2> "$out/bench.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o bench -- python3 bench.py --steps 10 --warmup 2 \
  --skip-node-configs > "$out/prof_bench.json" 2> "$out/prof_bench.err" || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d "$out/f32_pmc" -o run --output-format csv -- python3 tools/gemm_f32_pmc.py 256x256g8,256x256ir torch \
  > "$out/f32_pmc.log" 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$out/hostres" -o hr \
  -- python3 tools/hostres_probe.py 16 4 > "$out/hostres.json" 2> "$out/hostres.err" || exit $?
timeout -k 10 240 python tools/nbody_force_variants.py 1048576 1,0.25 "$out/nbody_variants.json" \
  > "$out/nbody_variants.log" 2>&1 || exit $?
timeout -k 10 240 python tools/gemm_f32_probe.py 8192 256x256g8,256x256g8@8,256x256g8@2,256x256g8@16 3 5 \
  > "$out/f32_gm.json" 2> "$out/f32_gm.err" || exit $?
[ -n "$CEK_SKIP_RANKS" ] && exit 0
timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --skip-node-configs --skip-mandelbrot \
  > "$out/bench_2r.json" 2> "$out/bench_2r.err" || exit $?
timeout -k 10 400 python bench.py --gpus 4 --size 4096 --steps 5 --warmup 2 --skip-node-configs --skip-mandelbrot \
  > "$out/bench_4r_4096.json" 2> "$out/bench_4r_4096.err" || exit $?
