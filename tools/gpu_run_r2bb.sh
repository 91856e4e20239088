source tools/gpu_steps.sh
step c3 300 python -u bench.py --config C3 --no-cpu-baseline -o gpurun_out/bench_bb_c3.json
step c4 300 python -u bench.py --config C4 --no-cpu-baseline -o gpurun_out/bench_bb_c4.json
step bal4 300 python -u tools/shard_balance.py --config C4 --split cost --worlds 8 > gpurun_out/bal_bb_c4.log 2>&1
step bal3 300 python -u tools/shard_balance.py --config C3 --split cost --worlds 4 > gpurun_out/bal_bb_c3.log 2>&1
grep "world\|full" gpurun_out/bal_bb_c4.log gpurun_out/bal_bb_c3.log
