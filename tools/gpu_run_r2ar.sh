source tools/gpu_steps.sh
step tests 600 python -u -m pytest tests/test_lbs_paths.py -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_ar.log 2>&1
tail -2 gpurun_out/gpu_tests_ar.log
step c5 300 python -u bench.py --config C5 --steps 120 -o gpurun_out/bench_ar_c5.json
