#!/bin/bash
# 2-rank gloo rehearsal of bench.py --shard rays on one card (graph-captured shards + all-gather), spawn tests.
source tools/gpu_steps.sh
export APN_DIST_BACKEND=gloo
step bench2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/zc_bench2.log 2>&1
unset APN_DIST_BACKEND
step spawn 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_0_shard_spawn.py tests/test_frame_graph.py > gpurun_out/zc_spawn.log 2>&1
