#!/bin/bash
# C5 LBS kernel HBM traffic: rocprofv3 kernel-trace stats + FETCH_SIZE / WRITE_SIZE in separate
# PMC passes over bench.py --config C5, summarised into profiles/<tag>_lbs_traffic_c5.json form.
# Usage (on the GPU box, from the repo root): tools/c5_traffic.sh <outdir> <tag>
set -o pipefail
OUT=${1:-gpurun_out/c5pmc}; TAG=${2:-r05}
ARGS="--config C5 --steps 40 --warmup 2 --no-cpu-baseline"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err" || exit $?
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/pmc$i" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/pmc$i.json" 2> "$OUT/pmc$i.err" || exit $?
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt" || exit 1
python3 - "$OUT/summary.txt" "$OUT/${TAG}_lbs_traffic_c5.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
name = next(k for k in d if "k_lbs_skin" in k)
e = d[name]
json.dump({"kernel": name, "bytes_per_launch": e["hbm_bytes_per_launch"], "avg_ms_profiled": e["avg_ms"],
           "FETCH_SIZE_KB": e["FETCH_SIZE"], "WRITE_SIZE_KB": e["WRITE_SIZE"],
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes (tools/c5_traffic.sh, bench.py "
                     "--config C5); bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024",
           "b_alg_per_launch": 216000000}, open(sys.argv[2], "w"), indent=1)
print(open(sys.argv[2]).read())
PY
