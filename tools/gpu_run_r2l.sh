source tools/gpu_steps.sh
export AB_STEPS=10
step tests 300 python -u -m pytest tests/test_hip_parity.py -m gpu -q -x -rf --timeout 200 --timeout-method thread -k "knn_modes" > gpurun_out/gpu_tests13.log 2>&1
tail -2 gpurun_out/gpu_tests13.log
step ab 900 bash tools/ab.sh "APN_KNN_MODE=8" "APN_KNN_MODE=9" "APN_KNN_MODE=9 APN_KNN_ANISO=4" "APN_KNN_MODE=9 APN_KNN_STATS=1" "APN_KNN_MODE=8 APN_KNN_STATS=1"
grep -h "knn" gpurun_out/ab/run4.err gpurun_out/ab/run5.err | head -20 || true
