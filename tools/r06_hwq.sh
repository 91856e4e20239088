#!/bin/bash
# C2 headline loop (4 frames in flight) with the HIP runtime's hardware queues per process at the
# box default (4) and at 8, interleaved.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
O=gpurun_out/r06q; mkdir -p $O
for r in 1 2 3; do for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 32 --warmup 3 --no-cpu-baseline --no-other-configs --no-viewpoints --no-full-mlp-leg -o $O/q_${q}_$r.json > /dev/null 2> $O/q_${q}_$r.err || { tail -20 $O/q_${q}_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/q_${q}_$r.json')); print('hw queues $q', '%.3f ms/frame' % d['ms_per_step'], 'serial %.3f' % d['config']['serial_ms_per_step'])"
done; done
