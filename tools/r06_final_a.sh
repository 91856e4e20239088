# Round-6 measurements, part A (outputs under gpurun_out/r06_final/): the GPU test suite, the
# default bench line and the C5 line. A fault / abort / timeout ends the call.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
O=gpurun_out/r06_final; mkdir -p $O
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?
  echo "[$name] rc=$rc"
  case $rc in 0|1) return 0;; *) tail -20 $O/$name.err; exit $rc;; esac
}
step gpu_tests 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -p no:cacheprovider
tail -3 $O/gpu_tests.out
step bench 400 python bench.py
tail -c 300 $O/bench.out; echo; grep -E "stage ms|in flight|render_viewpoints|other configs|full MLP" $O/bench.err
step c5 150 python bench.py --config C5 --steps 300
tail -c 300 $O/c5.out
