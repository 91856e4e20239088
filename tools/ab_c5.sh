#!/bin/bash
# C5 A/B: tools/ab_c5.sh "ENV=a" "ENV=b" ... (each arg: env assignments for one run)
set -o pipefail
mkdir -p gpurun_out/ab
i=0
for spec in "$@"; do
  i=$((i+1))
  env $spec timeout -k 10 240 python3 bench.py --config C5 --no-cpu-baseline --steps 60 --warmup 5 -o gpurun_out/ab/c5_$i.json 2> gpurun_out/ab/c5_$i.err || { echo "run $i ($spec) failed rc=$?"; tail -5 gpurun_out/ab/c5_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab/c5_$i.json'))
print('%-60s step %.4f ms  lbs %.4f ms  frac %.3f' % ('$spec', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac']))"
done
