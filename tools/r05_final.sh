# Round-5 closing measurements on one GPU (outputs under gpurun_out/r05_final/): GPU test suite,
# the default bench line, its rocprofv3 kernel stats, the PMC passes (raw output kept in /tmp, only
# the summaries returned), the training step and its kernel stats, the ray-shard balance and the
# 2-rank gloo rehearsal of the ray-sharded step on one card.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
O=gpurun_out/r05_final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
tail -3 $O/gpu_tests.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
tail -c 400 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-other-configs --no-viewpoints > $O/trace_bench.json 2> $O/trace_bench.err || exit 1
bash tools/pmc_profile.sh /tmp/r05pmc > $O/pmc.log 2>&1 || exit 1
cp /tmp/r05pmc/summary.txt $O/pmc_summary.txt && python3 tools/mlp_traffic.py $O/pmc_summary.txt $O/point_mlp_traffic.json "round-5 final state" || exit 1
timeout -k 10 200 python -u tools/train_bench.py --steps 30 --warmup 5 > $O/train.json 2> $O/train.err || exit 1
bash tools/train_rocprof.sh $O/tprof --steps 10 --warmup 3 --no-cpu-baseline || exit 1
timeout -k 10 300 python tools/shard_balance.py --split gilv4096 --worlds 2,4,8 --reps 10 --in-flight 3 > $O/shard_balance.log 2>&1 || exit 1
APN_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-other-configs --no-viewpoints > $O/gloo2.json 2> $O/gloo2.err || exit 1
# gpurun returns at most 64 MiB: keep the summaries, drop the per-dispatch traces
find $O -name "*kernel_trace.csv" -delete; find $O -name "*counter_collection.csv" -delete
find $O -name "*_trace.csv" -size +4M -delete
du -sh $O
echo done
