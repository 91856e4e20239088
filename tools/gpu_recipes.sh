#!/bin/bash
# Named GPU-box recipes (they replace round 2's one-off tools/gpu_run_r2*.sh scripts). Each step
# runs under its own time limit (tools/gpu_steps.sh) and the call stops at the first failure.
# Usage on the GPU box, from the repo root:  bash tools/gpu_recipes.sh <recipe>[,<recipe>...] [bench args]
#   tests    pytest -m gpu              -> gpurun_out/gpu_tests.log
#   smoke    __graft_entry__.smoke()
#   bench    bench.py (default C2 line) -> gpurun_out/bench.json   (extra args go to bench.py)
#   rocprof  rocprofv3 --kernel-trace --stats of the bench line -> gpurun_out/bprof/
#   pmc      PMC counter passes of the bench line (one pass per counter group) -> gpurun_out/pmc/
#   probe    multi-process determinism probe (tools/determinism_probe3.py) -> gpurun_out/probe3.log
source "$(dirname "$0")/gpu_steps.sh"
recipes=$1; shift
IFS=, read -ra list <<< "$recipes"
for r in "${list[@]}"; do
  case $r in
    tests)   step tests 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread \
                 > gpurun_out/gpu_tests.log 2>&1; tail -3 gpurun_out/gpu_tests.log ;;
    smoke)   step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)   step bench 400 python -u bench.py -o gpurun_out/bench.json "$@" ;;
    rocprof) step rocprof 400 bash tools/bench_rocprof.sh gpurun_out/bprof "$@" ;;
    pmc)     step pmc 900 bash tools/pmc_profile.sh gpurun_out/pmc "$@" ;;
    probe)   step probe 300 python -u tools/determinism_probe3.py 600 default 3 > gpurun_out/probe3.log 2>&1 ;;
    *) echo "unknown recipe $r"; exit 2 ;;
  esac
done
