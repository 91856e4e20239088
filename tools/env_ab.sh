#!/bin/bash
# A/B of environment settings on the C2 bench line (stage ms from HIP events), interleaved.
# Usage on the GPU box: ENVS="APN_KNN_MODE=9 APN_KNN_MODE=10" ROUNDS=2 bash tools/env_ab.sh [bench args]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
# the environment switches exist in the debug build only (include/apn_hip_debug.h)
export APN_HIP_LIB=${APN_HIP_LIB:-$PWD/articulated-point-nerf_amd/apn_amd/libapn_hip_debug.so}
i=0
for r in $(seq 1 ${ROUNDS:-2}); do for e in $ENVS; do
  i=$((i+1))
  env ${e//,/ } timeout -k 10 150 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-other-configs -o gpurun_out/envab_$i.json "$@" 2>/dev/null >/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/envab_$i.json')); s=d['stage_ms']; print('$e', 'mlp %.3f knn %.3f frame %.3f' % (s['mlp'], s['knn'], d['ms_per_step']))"
done; done
