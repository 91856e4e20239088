source tools/gpu_steps.sh
APN_MLP_GROUPS=3 step tests_g3 600 python -u -m pytest tests/test_mlp_precision.py tests/test_hip_parity.py -m gpu -q -x -rf --timeout 300 --timeout-method thread -k "mlp or forward or same_cloud" > gpurun_out/gpu_tests_u.log 2>&1
tail -3 gpurun_out/gpu_tests_u.log
AB_STEPS=20 step ab 600 bash tools/ab.sh "APN_AB=g1" "APN_MLP_GROUPS=3" "APN_AB=g1b" "APN_MLP_GROUPS=3"
