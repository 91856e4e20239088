#!/bin/bash
# A/B of libapn_hip variants (ab/<tag>/libapn_hip.so, tools/ab_build.sh) on the C2
# bench line: MLP kernel ms (HIP events) and frame ms, variants interleaved over ROUNDS rounds.
# Usage on the GPU box: VARIANTS="h3V0 h3V1" ROUNDS=2 bash tools/mlp_ab.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for r in $(seq 1 ${ROUNDS:-2}); do for v in $VARIANTS; do
  APN_HIP_LIB=$PWD/ab/$v/libapn_hip.so timeout -k 10 150 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-other-configs --no-viewpoints --no-full-mlp-leg -o gpurun_out/ab_$v.json 2>/dev/null >/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); s=d['stage_ms']; print('$v', 'mlp %.3f kernel %.3f knn %.3f frame %.3f serial %.3f' % (s['mlp'], d['roofline']['avg_launch_ms'], s['knn'], d['ms_per_step'], d['config'].get('serial_ms_per_step') or 0))"
done; done
