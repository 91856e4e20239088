cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in ${VARIANTS:-A}; do for bpc in ${BPCS:-4 6}; do
  APN_HIP_LIB=$PWD/articulated-point-nerf_amd/apn_amd/libapn_hip_lbs$v.so APN_LBS_BLOCKS_PER_CU=$bpc timeout -k 10 120 python bench.py --config C5 --steps 200 --warmup 20 --no-cpu-baseline -o gpurun_out/c5_$v$bpc.json 2>/dev/null >/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/c5_$v$bpc.json')); print('$v', $bpc, 'lbs_ms %.4f frac %.3f step_ms %.4f' % (d['config']['lbs_kernel_ms'], d['roofline']['frac'], d['ms_per_step']))"
done; done
