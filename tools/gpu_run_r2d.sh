source tools/gpu_steps.sh
step tests 600 python -u -m pytest tests/test_lbs_paths.py tests/test_tineuvox.py tests/test_hip_parity.py -m gpu -q -rf --timeout 300 --timeout-method thread -k "lbs or repose or tineuvox or vox or skeleton or pointwarper or grid or forward_vs or canonical or train" > gpurun_out/gpu_tests5.log 2>&1
tail -6 gpurun_out/gpu_tests5.log
step bench_c5 300 python -u bench.py --config C5 --steps 60 --warmup 5 > gpurun_out/bench5_c5.json 2> gpurun_out/bench5_c5.err
cat gpurun_out/bench5_c5.json
step bench_c2 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench5.json 2> gpurun_out/bench5.err
step bench_c2_r1 300 bash -c 'cd ab/r1 && python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline' > gpurun_out/bench5_r1.json 2> gpurun_out/bench5_r1.err
python3 - <<'PY'
import json
for f in ("gpurun_out/bench5.json", "gpurun_out/bench5_r1.json"):
    try:
        d = json.load(open(f)); print(f, round(d["ms_per_step"], 3), d["stage_ms"])
    except Exception as e: print(f, e)
PY
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step rocprof_c5 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --config C5 --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/bench5_c5_prof.json 2> gpurun_out/bench5_c5_prof.err
