#!/bin/bash
# A/B bench runs on the GPU box: tools/ab.sh "ENV=a" "ENV=b" ... (each arg: env assignments for one run)
# Prints one summary line per run: env, rays/s, ms/step, k_point_mlp ms.
set -o pipefail
mkdir -p gpurun_out/ab
i=0
for spec in "$@"; do
  i=$((i+1))
  env $spec timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-other-configs --steps ${AB_STEPS:-10} > gpurun_out/ab/run$i.json 2> gpurun_out/ab/run$i.err || { echo "run $i ($spec) failed rc=$?"; tail -5 gpurun_out/ab/run$i.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/ab/run$i.json'))
print('%-40s %.3fM rays/s  %.2f ms/step  mlp %.2f ms  stages %s' % ('$spec', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('stage_ms')))"
done
