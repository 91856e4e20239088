source tools/gpu_steps.sh
step tests 600 python -u -m pytest tests/test_hip_parity.py tests/test_frame_graph.py tests/test_0_shard_spawn.py -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_bd.log 2>&1
tail -1 gpurun_out/gpu_tests_bd.log
APN_CELL_BOUND16_MAX=100000000 step tests16 600 python -u -m pytest tests/test_hip_parity.py -m gpu -q -x -rf --timeout 300 --timeout-method thread -k "knn_modes or stagewise" > gpurun_out/gpu_tests_bd16.log 2>&1
tail -1 gpurun_out/gpu_tests_bd16.log
step bal 300 python -u tools/shard_balance.py --split cost --worlds 4,8 > gpurun_out/bal_bd.log 2>&1
grep "world\|full" gpurun_out/bal_bd.log
step train 300 python -u tools/train_bench.py --no-cpu-baseline --steps 20 > gpurun_out/train_bd.json 2>&1
tail -1 gpurun_out/train_bd.json | cut -c1-200
AB_STEPS=20 step ab 300 bash tools/ab.sh "APN_AB=c2"
