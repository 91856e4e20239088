#!/bin/bash
# Collect rocprofv3 kernel-trace stats + PMC counter passes for the bench workload.
# Usage (on the GPU box, from the repo root): tools/pmc_profile.sh <outdir> [bench args]
# Each counter group runs in its own pass (FETCH_SIZE and WRITE_SIZE cannot share a pass).
set -o pipefail
OUT=${1:-gpurun_out/pmc}; shift
ARGS=${@:-"--steps 2 --warmup 1 --in-flight 1 --no-cpu-baseline --no-other-configs --no-viewpoints --no-full-mlp-leg"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err" || exit $?
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/pmc$i" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/pmc$i.json" 2> "$OUT/pmc$i.err" || exit $?
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt"
cat "$OUT/summary.txt"
