set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_nbr_loss.py -k "gemm" -m gpu > gpurun_out/r05_gemm_tests.log 2>&1 || { tail -40 gpurun_out/r05_gemm_tests.log; exit 1; }
tail -2 gpurun_out/r05_gemm_tests.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_graph.py -m gpu > gpurun_out/r05_train_graph_tests.log 2>&1 || { tail -60 gpurun_out/r05_train_graph_tests.log; exit 1; }
tail -2 gpurun_out/r05_train_graph_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_hip_parity.py -k "train or feat_depth or frozen" -m gpu > gpurun_out/r05_train_tests.log 2>&1 || { tail -40 gpurun_out/r05_train_tests.log; exit 1; }
tail -2 gpurun_out/r05_train_tests.log
timeout -k 10 200 python -u tools/train_bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05_train_bench2.json 2> gpurun_out/r05_train_bench2.err && cat gpurun_out/r05_train_bench2.json
bash tools/train_rocprof.sh gpurun_out/r05_tprof3 --steps 10 --warmup 3 --no-cpu-baseline
