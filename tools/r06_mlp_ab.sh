# MLP change: parity first (stage tests, precision vs float64, ERT, the C2 every-ray frame), then a
# same-box A/B of ab/base (previous commit) against ab/<new> on the C2 line, interleaved; then the
# default bench line and the C5 line on the product library.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
O=gpurun_out/r06m; mkdir -p $O
NEW=${NEW:-"pkr"}
PT="python -u -m pytest -q --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu"
[ -n "$SKIP_PARITY" ] || ${PARITY_NEW:+env APN_HIP_LIB=$PWD/ab/${NEW%% *}/libapn_hip.so} timeout -k 10 500 $PT tests/test_mlp_precision.py tests/test_ert.py "tests/test_hip_parity.py::test_mlp_stage_vs_oracle" "tests/test_full_frame_parity.py::test_every_ray_vs_oracle[C2]" -k "not C3 and not C4" -s > $O/parity.log 2>&1
rc=$?; [ -n "$SKIP_PARITY" ] || grep -E "passed|failed|every ray" $O/parity.log | tail -5
case $rc in 0) ;; *) echo "stop rc $rc"; grep -E "Error|assert" $O/parity.log | head -20; exit $rc;; esac
for r in 1 2; do for v in ${BASE:-base} $NEW; do
  APN_HIP_LIB=$PWD/ab/$v/libapn_hip.so timeout -k 10 200 python bench.py --steps 32 --warmup 3 --no-cpu-baseline --no-other-configs --no-viewpoints --no-full-mlp-leg -o $O/ab_${v}_$r.json 2>$O/ab_${v}_$r.err >/dev/null || { tail -20 $O/ab_${v}_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab_${v}_$r.json')); s=d['stage_ms']; print('$v', 'mlp %.3f kernel %.3f frac %.3f knn %.3f frame %.3f serial %.3f sameview %.3f' % (s['mlp'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], s['knn'], d['ms_per_step'], d['config'].get('serial_ms_per_step') or 0, d['config'].get('same_view_ms_per_step') or 0))"
done; done
[ -n "$SKIP_TAIL" ] && exit 0
timeout -k 10 120 python bench.py --config C5 --steps 300 > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python -c "import json; d=json.load(open('$O/c5.json')); print('C5', d['value']/1e9, 'Gpts/s', d['ms_per_step'], 'ms/pose, lbs', d['config']['lbs_kernel_ms'], d['roofline']['frac'])"
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
tail -22 $O/bench.err
