#!/bin/bash
# Heavy-first kNN block order: parity (default and forced on every launch), shard emulation, full frame.
source tools/gpu_steps.sh
step parity 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_parity.py tests/test_0_shard_spawn.py -k "knn or shards or blocks or spawn or frame" > gpurun_out/zb_parity.log 2>&1
APN_KNN_LPT_MAX=1000000000 step parity_forced 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_parity.py -k "knn or frame or golden" > gpurun_out/zb_parity_forced.log 2>&1
step ilv 200 python -u tools/shard_balance.py --split ilv4096 --worlds 4,8 --reps 10 > gpurun_out/zb_ilv.log 2>&1
APN_KNN_LPT_MAX=0 step ilv_off 200 python -u tools/shard_balance.py --split ilv4096 --worlds 8 --reps 10 > gpurun_out/zb_ilv_off.log 2>&1
APN_KNN_LPT_MAX=1000000000 step full_on 200 python -u tools/shard_balance.py --split ilv4096 --worlds 2 --reps 10 > gpurun_out/zb_full_on.log 2>&1
