source tools/gpu_steps.sh
export AB_STEPS=10
step tests 300 python -u -m pytest tests/test_hip_parity.py -m gpu -q -x -rf --timeout 200 --timeout-method thread -k "knn_modes and (8 or 9)" > gpurun_out/gpu_tests14.log 2>&1
tail -2 gpurun_out/gpu_tests14.log
step ab 900 bash tools/ab.sh "APN_KNN_MODE=9" "APN_KNN_MODE=9 APN_KNN_PTS=4" "APN_KNN_MODE=9 APN_KNN_A_ANISO=1" "APN_KNN_MODE=9 APN_KNN_SUBDIV=6" "APN_KNN_MODE=9 APN_KNN_SUBDIV=10"
export APN_KNN_MODE=9
step prof 300 bash tools/bench_rocprof.sh gpurun_out/bprof14 --steps 10 --warmup 3 --no-cpu-baseline
