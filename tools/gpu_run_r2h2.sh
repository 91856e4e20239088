source tools/gpu_steps.sh
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench 400 python -u bench.py --no-cpu-baseline --steps 20 -o gpurun_out/r2h2.json
