source tools/gpu_steps.sh
step t 300 python -u -m pytest tests/test_harness_gpu.py -q -x -rf --timeout 200 --timeout-method thread > gpurun_out/t_ag.log 2>&1
tail -2 gpurun_out/t_ag.log
APN_KNN_B9S=4 step t4 300 python -u -m pytest tests/test_hip_parity.py -q -x -rf --timeout 200 --timeout-method thread -k "knn_modes or stagewise" > gpurun_out/t_ag4.log 2>&1
tail -2 gpurun_out/t_ag4.log
APN_KNN_B9S=2 step bal2 300 python -u tools/shard_balance.py --split cost --worlds 4,8 > gpurun_out/bal_ag2.log 2>&1
APN_KNN_B9S=4 step bal4 300 python -u tools/shard_balance.py --split cost --worlds 4,8 > gpurun_out/bal_ag4.log 2>&1
step bal1 300 python -u tools/shard_balance.py --split cost --worlds 4,8 > gpurun_out/bal_ag1.log 2>&1
grep "world\|full" gpurun_out/bal_ag1.log gpurun_out/bal_ag2.log gpurun_out/bal_ag4.log
AB_STEPS=20 step ab 600 bash tools/ab.sh "APN_AB=base" "APN_HIP_LIB=ab/bpf1/libapn_hip.so" "APN_AB=base2" "APN_HIP_LIB=ab/bpf1/libapn_hip.so"
