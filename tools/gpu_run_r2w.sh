#!/bin/bash
# Blocks split: GPU parity (spawn + assemble tests), shard emulation through the model path.
source tools/gpu_steps.sh
step spawn 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_0_shard_spawn.py > gpurun_out/w_spawn.log 2>&1
step parity 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_parity.py -k "shards or blocks or chunk" > gpurun_out/w_parity.log 2>&1
step ilv 400 python -u tools/shard_balance.py --split cost,ilv2048,ilv4096,ilv8192 --worlds 2,4,8 --reps 5 > gpurun_out/w_ilv.log 2>&1
