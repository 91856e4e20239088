#!/bin/bash
# Blocks split + per-rank graph: spawn test (3 variants), frame-graph tests, blocks parity, bench.
source tools/gpu_steps.sh
step spawn 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_0_shard_spawn.py > gpurun_out/x_spawn.log 2>&1
step graphs 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_frame_graph.py tests/test_hip_parity.py -k "graph or captured or blocks or shards" > gpurun_out/x_tests.log 2>&1
step bench 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/x_bench.log 2>&1
