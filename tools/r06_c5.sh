# C5 repose step: the repose-sweep tests, then the three captured-step modes interleaved.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
O=gpurun_out/r06c5; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_lbs_paths.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; case $rc in 0) ;; *) grep -E "Error|assert" $O/tests.log | head; exit $rc;; esac
for r in 1 2; do for m in batched per_pose; do
  timeout -k 10 120 python bench.py --config C5 --steps 300 --no-cpu-baseline --repose-mode $m > $O/c5_${m}_$r.json 2> $O/c5_${m}_$r.err || { tail $O/c5_${m}_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c5_${m}_$r.json')); print('$m', round(d['value']/1e9,2), 'Gpts/s', round(d['ms_per_step'],4), 'ms/pose, lbs', round(d['config']['lbs_kernel_ms'],4), round(d['roofline']['frac'],3))"
done; done
