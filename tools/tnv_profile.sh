#!/bin/bash
# rocprofv3 kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes of tools/tineuvox_bench.py.
# Usage (GPU box, repo root): tools/tnv_profile.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/tnvprof}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 tools/tineuvox_bench.py --reps 5 > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err" || exit $?
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/pmc$i" -o run --output-format csv -- python3 tools/tineuvox_bench.py --reps 2 > "$OUT/pmc$i.json" 2> "$OUT/pmc$i.err" || exit $?
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt"
