#!/bin/bash
# C2 frames in flight 3 vs 4 on one box, interleaved twice (the headline loop only).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
O=gpurun_out/r06f; mkdir -p $O
for r in ${RS:-1 2}; do for n in ${NS:-3 4}; do
  timeout -k 10 200 python bench.py --steps 32 --warmup 3 --in-flight $n --no-cpu-baseline --no-other-configs --no-viewpoints --no-full-mlp-leg -o $O/f_${n}_$r.json > /dev/null 2> $O/f_${n}_$r.err || { tail -20 $O/f_${n}_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/f_${n}_$r.json')); print('in flight $n', '%.3f ms/frame' % d['ms_per_step'], '%.1f M rays/s' % (d['value']/1e6))"
done; done
