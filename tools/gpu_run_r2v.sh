source tools/gpu_steps.sh
step tests 600 python -u -m pytest tests/test_frame_graph.py tests/test_hip_parity.py tests/test_0_shard_spawn.py -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_v.log 2>&1
tail -3 gpurun_out/gpu_tests_v.log
AB_STEPS=20 step ab 600 bash tools/ab.sh "APN_AB=conc" "APN_CONCURRENT_GRID=0" "APN_AB=conc2" "APN_CONCURRENT_GRID=0"
