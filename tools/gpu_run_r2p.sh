source tools/gpu_steps.sh
step tests 400 python -u -m pytest tests/test_lbs_paths.py tests/test_hip_parity.py -m gpu -q -x -rf --timeout 200 --timeout-method thread -k "lbs or repose" > gpurun_out/gpu_tests17.log 2>&1
tail -2 gpurun_out/gpu_tests17.log
step bench_c5 300 python -u bench.py --config C5 --steps 60 --warmup 5 --no-cpu-baseline -o gpurun_out/bench17_c5.json
python3 -c "import json; d=json.load(open('gpurun_out/bench17_c5.json')); print(d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
