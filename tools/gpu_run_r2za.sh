#!/bin/bash
# kNN knobs on the 8-way blocks shards (one-GPU emulation).
source tools/gpu_steps.sh
step def 200 python -u tools/shard_balance.py --split ilv4096 --worlds 8 --reps 10 > gpurun_out/za_def.log 2>&1
APN_KNN_PTS=2 step pts2 200 python -u tools/shard_balance.py --split ilv4096 --worlds 8 --reps 10 > gpurun_out/za_pts2.log 2>&1
APN_KNN_ANISO=4 step an4 200 python -u tools/shard_balance.py --split ilv4096 --worlds 8 --reps 10 > gpurun_out/za_an4.log 2>&1
APN_KNN_ANISO=1 step an1 200 python -u tools/shard_balance.py --split ilv4096 --worlds 8 --reps 10 > gpurun_out/za_an1.log 2>&1
APN_KNN_B_SPLIT=1 step bsplit 200 python -u tools/shard_balance.py --split ilv4096 --worlds 8 --reps 10 > gpurun_out/za_bsplit.log 2>&1
APN_KNN_A_ANISO=1 step aan 200 python -u tools/shard_balance.py --split ilv4096 --worlds 8 --reps 10 > gpurun_out/za_aan.log 2>&1
