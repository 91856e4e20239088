source tools/gpu_steps.sh
step bench_c2_off 400 python -u bench.py --no-cpu-baseline --steps 20 --warmup 3 -o gpurun_out/r2y_c2_off.json
step bench_c2_on 400 python -u bench.py --no-cpu-baseline --steps 20 --warmup 3 --graph on -o gpurun_out/r2y_c2_on.json
step g3_full_repack 150 python -u tools/graph_diag.py --scene G3 --mode replay_only --full-repack
