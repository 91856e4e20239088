source tools/gpu_steps.sh
step tests 600 python -u -m pytest tests/test_lbs_paths.py tests/test_hip_parity.py -m gpu -q -x -rf --timeout 300 --timeout-method thread -k "repose or skeleton or lbs or weights" > gpurun_out/gpu_tests_aq.log 2>&1
tail -2 gpurun_out/gpu_tests_aq.log
step c5 300 python -u bench.py --config C5 -o gpurun_out/bench_aq_c5.json
