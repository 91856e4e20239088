source tools/gpu_steps.sh
step shard_tests 400 python -u -m pytest tests/test_0_shard_spawn.py tests/test_frame_graph.py -x -v --timeout 300 --timeout-method thread
step bench_gloo2 400 env APN_DIST_BACKEND=gloo python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --no-cpu-baseline --steps 10 -o gpurun_out/r2s_gloo2.json
