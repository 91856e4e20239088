set -o pipefail
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_parity.py -k "quad_lbs or lbs" tests/test_lbs_paths.py -m gpu > gpurun_out/r05_lbs_mfma_tests.log 2>&1 || { tail -30 gpurun_out/r05_lbs_mfma_tests.log; exit 1; }
tail -2 gpurun_out/r05_lbs_mfma_tests.log
D=$PWD/articulated-point-nerf_amd/apn_amd/libapn_hip_debug.so
bash tools/ab_c5.sh "APN_HIP_LIB=$D APN_LBS_QUAD=1" "APN_HIP_LIB=$D APN_LBS_BLOCKS_PER_CU=8" "APN_HIP_LIB=$D APN_LBS_BLOCKS_PER_CU=4" "APN_HIP_LIB=$D APN_LBS_BLOCKS_PER_CU=16" "APN_HIP_LIB=$PWD/ab/pf2w4/libapn_hip.so APN_LBS_BLOCKS_PER_CU=8" "APN_HIP_LIB=$PWD/ab/pf2w4/libapn_hip.so APN_LBS_BLOCKS_PER_CU=4" "APN_HIP_LIB=$D APN_LBS_QUAD=1" "APN_HIP_LIB=$D APN_LBS_BLOCKS_PER_CU=8" || exit 1
timeout -k 10 300 python -u tools/viewpoints_probe.py > gpurun_out/r05_vp_nf.log 2>&1
timeout -k 10 200 python -u tools/train_bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05_train_bench.json 2> gpurun_out/r05_train_bench.err && cat gpurun_out/r05_train_bench.json
bash tools/train_rocprof.sh gpurun_out/r05_tprof --steps 10 --warmup 3 --no-cpu-baseline
