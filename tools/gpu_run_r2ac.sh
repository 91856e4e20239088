source tools/gpu_steps.sh
APN_KNN_A_SPLIT=1 step tests 600 python -u -m pytest tests/test_hip_parity.py tests/test_frame_graph.py -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_ac.log 2>&1
tail -2 gpurun_out/gpu_tests_ac.log
AB_STEPS=20 step ab 600 bash tools/ab.sh "APN_AB=base" "APN_KNN_A_SPLIT=1" "APN_COMPOSITE=seq" "APN_AB=base2" "APN_KNN_A_SPLIT=1" "APN_COMPOSITE=seq"
