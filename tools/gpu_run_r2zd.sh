#!/bin/bash
# Blocks split shard emulation for C3 (4 shards) and C4 (8 shards).
source tools/gpu_steps.sh
step c3 300 python -u tools/shard_balance.py --config C3 --split cost,ilv4096 --worlds 4 --reps 5 > gpurun_out/zd_c3.log 2>&1
step c4 400 python -u tools/shard_balance.py --config C4 --split cost,ilv4096 --worlds 8 --reps 5 > gpurun_out/zd_c4.log 2>&1
