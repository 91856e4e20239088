#!/bin/bash
# C5 (LBS-only repose sweep, 1M points, 48 bones): poses in flight 1 / 2 / 3, interleaved twice on
# one box, after the repose-sweep tests (batched2 = two poses in flight).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
O=gpurun_out/r06c5; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 -p no:cacheprovider -m gpu tests/test_lbs_paths.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do for n in ${NS:-1 2 3}; do
  timeout -k 10 120 python bench.py --config C5 --steps 600 --warmup 5 --no-cpu-baseline --repose-in-flight $n > $O/c5_${n}_$r.json 2> $O/c5_${n}_$r.err || { tail -20 $O/c5_${n}_$r.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/c5_${n}_$r.json').read().strip().splitlines()[-1]); print('in flight $n', '%.2f G pts/s' % (d['value']/1e9), '%.4f ms/pose' % d['ms_per_step'], 'lbs %.4f' % d['config']['lbs_kernel_ms'])"
done; done
