source tools/gpu_steps.sh
step tests 900 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s.log 2>&1
tail -3 gpurun_out/gpu_tests_s.log
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python -u bench.py -o gpurun_out/bench_s.json
step bench_c5 300 python -u bench.py --config C5 --no-cpu-baseline -o gpurun_out/bench_s_c5.json
step rocprof 400 bash tools/bench_rocprof.sh gpurun_out/prof_s
