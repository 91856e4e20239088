source tools/gpu_steps.sh
step tnv 300 python -u tools/tineuvox_bench.py --reps 20
step tnv_prof 700 bash tools/tnv_profile.sh gpurun_out/r02_tnv
head -c 3000 gpurun_out/r02_tnv/summary.txt
step c2prof 400 bash tools/bench_rocprof.sh gpurun_out/r02_c2 --steps 10 --warmup 3 --no-cpu-baseline
step c5prof 300 bash -c 'cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r02_c5 && timeout -k 10 280 rocprofv3 --kernel-trace --stats -d gpurun_out/r02_c5/trace -o run --output-format csv -- python3 bench.py --config C5 --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/r02_c5/bench.json 2> gpurun_out/r02_c5/bench.err'
