source tools/gpu_steps.sh
APN_KNN_A_PTS=4 step t 300 python -u -m pytest tests/test_hip_parity.py -q -x -rf --timeout 200 --timeout-method thread -k "knn_modes or stagewise" > gpurun_out/t_ap.log 2>&1
tail -1 gpurun_out/t_ap.log
AB_STEPS=20 step ab 600 bash tools/ab.sh "APN_AB=base" "APN_KNN_A_PTS=4" "APN_AB=base2" "APN_KNN_A_PTS=4"
