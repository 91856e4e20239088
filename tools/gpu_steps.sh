#!/bin/bash
# Sourced by tools/gpu_recipes.sh on the GPU box.
#   step <name> <seconds> <command...>
# runs one GPU step under its own time limit and ends the script on any failure
# (fault, abort, time limit): no further GPU step runs in that call.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
step() {
  local name=$1 secs=$2; shift 2
  local t0=$(date +%s)
  echo "[step $name] start (limit ${secs}s)"
  timeout -k 10 "$secs" "$@"
  local rc=$?
  echo "[step $name] rc=$rc after $(( $(date +%s) - t0 ))s"
  if [ $rc -ne 0 ]; then
    echo "[step $name] FAILED: stopping this call"
    exit $rc
  fi
}
