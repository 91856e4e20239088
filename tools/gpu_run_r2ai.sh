source tools/gpu_steps.sh
step tests 900 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_ai.log 2>&1
tail -2 gpurun_out/gpu_tests_ai.log
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python -u bench.py --no-cpu-baseline -o gpurun_out/bench_ai.json
step ilv 200 python -u tools/shard_balance.py --split ilv4096 --worlds 2,4,8 --reps 10 > gpurun_out/ai_ilv.log 2>&1
