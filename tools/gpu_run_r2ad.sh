source tools/gpu_steps.sh
step tests 600 python -u -m pytest tests/test_hip_parity.py tests/test_frame_graph.py -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_ad.log 2>&1
tail -2 gpurun_out/gpu_tests_ad.log
AB_STEPS=20 step ab 600 bash tools/ab.sh "APN_AB=base" "APN_CELL_BOUND=thread" "APN_AB=base2" "APN_CELL_BOUND=thread"
