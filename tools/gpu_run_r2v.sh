#!/bin/bash
# Interleaved-block ray shards vs the cost split, one-GPU emulation.
source tools/gpu_steps.sh
step ilv 400 python -u tools/shard_balance.py --split cost,ilv64,ilv800,ilv4096 --worlds 4,8 --reps 5 > gpurun_out/ilv.log 2>&1
