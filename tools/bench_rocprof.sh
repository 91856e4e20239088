#!/bin/bash
# rocprofv3 kernel-trace stats of the default bench.py line (C2 render).
# Usage (on the GPU box, from the repo root): tools/bench_rocprof.sh <outdir> [bench args]
set -o pipefail
OUT=${1:-gpurun_out/bprof}; shift
ARGS=${@:-"--steps 10 --warmup 3 --no-cpu-baseline --no-other-configs"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
