source tools/gpu_steps.sh
step stats_mask 300 env APN_KNN_STATS=1 python -u bench.py --no-cpu-baseline --steps 5 --warmup 1 --graph off -o gpurun_out/r2m2_a.json
step stats_nomask 300 env APN_KNN_STATS=1 APN_KNN_MASK=0 python -u bench.py --no-cpu-baseline --steps 5 --warmup 1 --graph off -o gpurun_out/r2m2_b.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step prof_mask 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mask -o run -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 --graph off
