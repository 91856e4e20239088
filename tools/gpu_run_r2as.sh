source tools/gpu_steps.sh
step tests 600 python -u -m pytest tests/test_lbs_paths.py -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_as.log 2>&1
tail -1 gpurun_out/gpu_tests_as.log
step ab 300 python -u tools/c5_step_ab.py
