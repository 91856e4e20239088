#!/bin/bash
# rocprof A/B of libapn_hip variants (ab/<tag>/libapn_hip.so): per-kernel average us of the kNN
# kernels on the C2 bench line, variants interleaved over ROUNDS rounds.
# Usage on the GPU box: VARIANTS="a b" ROUNDS=2 bash tools/knn_prof_ab.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for r in $(seq 1 ${ROUNDS:-2}); do for v in $VARIANTS; do
  APN_HIP_LIB=$PWD/ab/$v/libapn_hip.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/kp_${v}_$r -o run \
    --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-other-configs > /dev/null 2>&1 || exit 1
  python3 - "$v" "gpurun_out/kp_${v}_$r" <<'PY'
import csv, glob, os, sys
KERNELS = os.environ.get("KERNELS")
f = glob.glob(sys.argv[2] + "/**/run_kernel_stats.csv", recursive=True)[0]
out = []
for r in csv.DictReader(open(f)):
    n = r["Name"].split("(")[0]
    if any(k in n for k in (KERNELS or "knn_pass cell_bound point_mlp").split()):
        out.append("%s %.1f" % (n.split("::")[-1][:22], float(r["AverageNs"]) / 1e3))
print(sys.argv[1], " | ".join(out))
PY
done; done
