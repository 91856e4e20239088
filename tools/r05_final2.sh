# Round-5 closing measurements after the MLP operand-read pinning (outputs under $O, default gpurun_out/r05_final4/):
# GPU test suite, the default bench line, its rocprofv3 kernel stats, the PMC passes (raw output in
# /tmp, only the summaries returned) and the ray-shard balance. The training step does not run the
# neighbour-MLP kernel (its numbers stay those of tools/r05_final.sh).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
O=${O:-gpurun_out/r05_final4}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
tail -3 $O/gpu_tests.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
tail -c 400 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-other-configs --no-viewpoints > $O/trace_bench.json 2> $O/trace_bench.err || exit 1
bash tools/pmc_profile.sh /tmp/r05pmc > $O/pmc.log 2>&1 || exit 1
cp /tmp/r05pmc/summary.txt $O/pmc_summary.txt && python3 tools/mlp_traffic.py $O/pmc_summary.txt $O/point_mlp_traffic.json "round-5 closing state (operand reads pinned, one launch per pass)" || exit 1
timeout -k 10 300 python tools/shard_balance.py --split gilv4096 --worlds 2,4,8 --reps 10 --in-flight 3 > $O/shard_balance.log 2>&1 || exit 1
find $O -name "*kernel_trace.csv" -delete; find $O -name "*counter_collection.csv" -delete
find $O -name "*_trace.csv" -size +4M -delete
du -sh $O
echo done
