source tools/gpu_steps.sh
step spawn 300 python -u -m pytest tests/test_0_shard_spawn.py tests/test_frame_graph.py -m gpu -q -x -rf --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_x.log 2>&1
tail -3 gpurun_out/gpu_tests_x.log
step bal 300 python -u tools/shard_balance.py
