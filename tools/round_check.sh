#!/bin/bash
# One GPU call that re-validates a fresh tree: GPU tests, smoke, the 1-GPU
# bench, a 2-rank bench rehearsal on the one GPU (gloo control plane, both
# ranks on GPU 0) and a rocprofv3 kernel trace of a short bench run.
# usage (from the repo root, via gpurun): bash tools/round_check.sh [steps...]
# steps default to: tests smoke bench bench2 prof  (also: bench4, bench8r)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
steps=("$@")
[ ${#steps[@]} -eq 0 ] && steps=(tests smoke bench bench2 prof)
specs=()
for s in "${steps[@]}"; do
  case "$s" in
    tests)  specs+=("gpu_tests:900:python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread") ;;
    smoke)  specs+=("smoke:180:python -c 'import __graft_entry__ as g; g.smoke()'") ;;
    bench)  specs+=("bench1:300:python bench.py") ;;
    bench2) specs+=("bench2:400:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2") ;;
    # bench.py starts the ranks itself, default tile (4 ranks: 256x256pb, one wave of tiles each)
    bench4) specs+=("bench4:500:python bench.py --gpus 4 --steps 10 --warmup 2") ;;
    # bench.py starts the ranks itself (no torchrun environment): 8 ranks on the one GPU
    bench8r) specs+=("bench8r:500:python bench.py --gpus 8 --steps 10 --warmup 2 --tile 256x256pb --skip-node-configs") ;;
    prof)   specs+=("prof:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 10 --warmup 2 && python tools/summarize_prof.py gpurun_out/prof_bench 'bench.py kernel trace (1 GPU, 10 steps)' > gpurun_out/prof_bench.md") ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
bash tools/gpu_session.sh "${specs[@]}"
