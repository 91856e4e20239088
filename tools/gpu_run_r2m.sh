source tools/gpu_steps.sh
step knn_tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "knn or forward or frame or smoke"
step bench_mask 300 python -u bench.py --no-cpu-baseline --steps 20 -o gpurun_out/r2m_mask.json
step bench_nomask 300 env APN_KNN_MASK=0 python -u bench.py --no-cpu-baseline --steps 20 -o gpurun_out/r2m_nomask.json
