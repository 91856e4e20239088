source tools/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step debug_band 300 python -u tools/debug_band.py C3 rgb_marched_direct > gpurun_out/debug_band.log 2>&1
step tests 600 python -u -m pytest tests/test_mlp_precision.py tests/test_hip_parity.py -m gpu -q -rf --timeout 300 --timeout-method thread -k "precision or sticky or band or mlp_stage" > gpurun_out/gpu_tests3.log 2>&1
step rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2b -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench3.json 2> gpurun_out/bench3.err
tail -8 gpurun_out/gpu_tests3.log; cat gpurun_out/bench3.json
