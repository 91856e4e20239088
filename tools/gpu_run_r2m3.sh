source tools/gpu_steps.sh
step knn_tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "knn or forward_vs or frame"
step stats_mask 300 env APN_KNN_STATS=1 python -u bench.py --no-cpu-baseline --steps 5 --warmup 1 --graph off -o gpurun_out/r2m3_a.json
step bench_mask 300 python -u bench.py --no-cpu-baseline --steps 20 -o gpurun_out/r2m3_mask.json
step bench_nomask 300 env APN_KNN_MASK=0 python -u bench.py --no-cpu-baseline --steps 20 -o gpurun_out/r2m3_nomask.json
