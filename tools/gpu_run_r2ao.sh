source tools/gpu_steps.sh
step tests 600 python -u -m pytest tests/test_hip_parity.py tests/test_nbr_loss.py -m gpu -q -x -rf --timeout 300 --timeout-method thread -k "train or autograd or loss or optimizer" > gpurun_out/gpu_tests_ao.log 2>&1
tail -2 gpurun_out/gpu_tests_ao.log
step train 300 python -u tools/train_bench.py --no-cpu-baseline --steps 20 > gpurun_out/train_ao.json 2>&1
tail -1 gpurun_out/train_ao.json
