# Round 6 measurements: the default bench line (16 distinct views), the C5 line, and a serial
# (--in-flight 1) rocprofv3 kernel trace of the C2 frame. Each step under its own time limit.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
O=gpurun_out/r06b; mkdir -p $O
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
tail -25 $O/bench.err; tail -c 600 $O/bench.json
timeout -k 10 200 python bench.py --config C5 --steps 300 > $O/c5.json 2> $O/c5.err || { tail -30 $O/c5.err; exit 1; }
tail -c 500 $O/c5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 16 --warmup 3 --in-flight 1 --no-cpu-baseline --no-other-configs --no-viewpoints --no-full-mlp-leg > $O/trace_bench.json 2> $O/trace_bench.err || exit 1
find $O -name "*kernel_trace.csv" -delete
find $O -name "*kernel_stats.csv" | head -3
