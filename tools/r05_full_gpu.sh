set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu > gpurun_out/r05_full_gpu.log 2>&1 || { tail -40 gpurun_out/r05_full_gpu.log; exit 1; }
tail -3 gpurun_out/r05_full_gpu.log
timeout -k 10 200 python -u tools/train_bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r05_train_bench3.json 2> gpurun_out/r05_train_bench3.err && cat gpurun_out/r05_train_bench3.json
