source tools/gpu_steps.sh
step bal 300 python -u tools/shard_balance.py --split inbbox,cost --worlds 2,4,8 > gpurun_out/bal_z.log 2>&1
grep "world\|full" gpurun_out/bal_z.log
APN_KNN_SMALL_MAX=131072 step bal2 300 python -u tools/shard_balance.py --split cost --worlds 8 > gpurun_out/bal_z2.log 2>&1
grep "world" gpurun_out/bal_z2.log
step train 300 python -u tools/train_bench.py --no-cpu-baseline > gpurun_out/train_z.log 2>&1
tail -2 gpurun_out/train_z.log
APN_KNN_SMALL_MAX=1048576 step train_old 300 python -u tools/train_bench.py --no-cpu-baseline > gpurun_out/train_z2.log 2>&1
tail -2 gpurun_out/train_z2.log
