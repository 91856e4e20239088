source tools/gpu_steps.sh
step spawn 300 python -u -m pytest tests/test_0_shard_spawn.py -m gpu -q -x -rf --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_aa.log 2>&1
tail -2 gpurun_out/gpu_tests_aa.log
APN_DIST_BACKEND=gloo step rehearse2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 8 --warmup 4 --no-cpu-baseline > gpurun_out/reh2.json 2> gpurun_out/reh2.err
cat gpurun_out/reh2.json; grep "rank\|Error" gpurun_out/reh2.err | tail -6
