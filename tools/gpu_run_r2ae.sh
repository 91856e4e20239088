source tools/gpu_steps.sh
step bench 300 python -u bench.py -o gpurun_out/bench_ae.json
step bench_c5 300 python -u bench.py --config C5 -o gpurun_out/bench_ae_c5.json
step rocprof 400 bash tools/bench_rocprof.sh gpurun_out/prof_ae
step pmc 900 bash tools/pmc_profile.sh gpurun_out/pmc_ae
