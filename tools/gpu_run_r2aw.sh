source tools/gpu_steps.sh
step bench 300 python -u bench.py -o gpurun_out/bench_aw.json
step rocprof 400 bash tools/bench_rocprof.sh gpurun_out/prof_aw
step pmc 900 bash tools/pmc_profile.sh gpurun_out/pmc_aw
