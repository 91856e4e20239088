#!/bin/bash
# Blocks split shards: eager vs per-rank graph replay, one-GPU emulation.
source tools/gpu_steps.sh
step ilv 400 python -u tools/shard_balance.py --split ilv4096,gilv4096 --worlds 2,4,8 --reps 10 > gpurun_out/y_ilv.log 2>&1
