# round-4 shard diagnostics (one GPU): kNN pass-B variants on a ray shard of 8 and on the full frame
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
DBG=articulated-point-nerf_amd/apn_amd/libapn_hip_debug.so
for P in 4 8; do for W in 8 1; do APN_HIP_LIB=$DBG APN_KNN_PTS=$P timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/spP${P}w$W -o run --output-format csv -- python3 tools/shard_profile.py --world $W > gpurun_out/spP${P}w$W.log 2>&1 || exit 1; done; done
echo done
