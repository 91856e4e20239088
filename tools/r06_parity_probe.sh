# Round 6 GPU call: the pipeline / repose sweep tests, the training-graph tests (AccumulateGrad
# warning as an error), the AccumulateGrad probe, the C3/C4 every-ray and ERT full-frame parity
# tests, and last tools/graph_capture_probe.py --only transformnet.
# A step that faults, aborts or times out ends the call (no further GPU work).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
O=gpurun_out/r06; mkdir -p $O
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "[$name] rc=$rc"; tail -4 $O/$name.log
  case $rc in 0|1) return 0;; *) echo "stopping after $name (rc $rc)"; exit $rc;; esac
}
PT="python -u -m pytest -v --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu -s"
run pipeline_lbs 400 $PT tests/test_pipeline.py tests/test_lbs_paths.py
run train 400 $PT tests/test_train_graph.py tests/test_hip_parity.py -k "train or training or G1"
run accgrad_probe 300 python -u tools/accumulate_grad_probe.py
run parity_c34 900 $PT tests/test_ert.py tests/test_full_frame_parity.py
grep -E "every ray|kept [0-9]|passed|failed|Error" $O/parity_c34.log | tail -30
run capture_probe 200 python -u tools/graph_capture_probe.py --only transformnet
