source tools/gpu_steps.sh
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step ab_c5 600 bash tools/ab_c5.sh "APN_AB=cur" "APN_HIP_LIB=ab/nopf/libapn_hip.so" "APN_AB=cur2" "APN_HIP_LIB=ab/nopf/libapn_hip.so"
step g3_replay_only 150 python -u tools/graph_diag.py --scene G3 --mode replay_only
step g3_bench_like 150 python -u tools/graph_diag.py --scene G3 --mode bench_like
step c2_bench_like 200 python -u tools/graph_diag.py --scene C2 --mode bench_like
