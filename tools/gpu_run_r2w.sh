source tools/gpu_steps.sh
step g3_bench_like 150 python -u tools/graph_diag.py --scene G3 --mode bench_like
step c2_replay_only 150 python -u tools/graph_diag.py --scene C2 --mode replay_only
step c2_bench_like 150 python -u tools/graph_diag.py --scene C2 --mode bench_like
