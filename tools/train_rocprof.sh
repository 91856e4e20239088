#!/bin/bash
# rocprofv3 kernel-trace stats of the train_pcd step (tools/train_bench.py).
# Usage (on the GPU box, from the repo root): tools/train_rocprof.sh <outdir> [train_bench args]
set -o pipefail
OUT=${1:-gpurun_out/tprof}; shift
ARGS=${@:-"--steps 10 --warmup 3 --no-cpu-baseline --no-other-configs"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 tools/train_bench.py $ARGS > "$OUT/train.json" 2> "$OUT/train.err" || exit $?
