# Helper for GPU calls: `step NAME TIMEOUT CMD...` runs one GPU step under its own time limit and
# stops the whole call on a crash / abort / time limit (rc >= 124 or a signal); test failures
# (rc 1) and usage errors (rc 2..) let the call continue. Source from a gpurun command script.
set -o pipefail
mkdir -p gpurun_out
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name"
  timeout -k 10 "$lim" "$@"
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ]; then echo "== stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
