source tools/gpu_steps.sh
step tests 600 python -u -m pytest tests/test_tineuvox.py tests/test_0_shard_spawn.py tests/test_mlp_precision.py tests/test_hip_parity.py -m gpu -q -rf --timeout 300 --timeout-method thread -k "tineuvox or spawn or precision or sticky or band or mlp_stage or vox or forward or grid or canonical" > gpurun_out/gpu_tests4.log 2>&1
tail -15 gpurun_out/gpu_tests4.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2c -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench4.json 2> gpurun_out/bench4.err
cat gpurun_out/bench4.json
