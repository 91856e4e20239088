source tools/gpu_steps.sh
step tests 900 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_ah.log 2>&1
tail -2 gpurun_out/gpu_tests_ah.log
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python -u bench.py --no-cpu-baseline -o gpurun_out/bench_ah.json
