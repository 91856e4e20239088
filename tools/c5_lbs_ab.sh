#!/bin/bash
# C5 LBS A/B of library builds (ab/<tag>/libapn_hip.so, tools/ab_build.sh) x blocks per CU.
# (APN_LBS_BLOCKS_PER_CU is read by debug builds only: build the variants with -DAPN_DEBUG_BUILD)
# Usage on the GPU box: VARIANTS="base x" BPCS="8 32" bash tools/c5_lbs_ab.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in ${VARIANTS:-base}; do for bpc in ${BPCS:-32}; do
  APN_HIP_LIB=$PWD/ab/$v/libapn_hip.so APN_LBS_BLOCKS_PER_CU=$bpc timeout -k 10 120 python bench.py --config C5 --steps 200 --warmup 20 --no-cpu-baseline -o gpurun_out/c5_$v$bpc.json 2>/dev/null >/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/c5_$v$bpc.json')); print('$v', $bpc, 'lbs_ms %.4f frac %.3f step_ms %.4f' % (d['config']['lbs_kernel_ms'], d['roofline']['frac'], d['ms_per_step']))"
done; done
