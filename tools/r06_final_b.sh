# Round-6 measurements, part B: PMC passes (serial), the serial rocprofv3 kernel stats, the
# ray-shard balance and the 2-rank gloo rehearsal of the ray-sharded step on one card.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
O=gpurun_out/r06_final; mkdir -p $O
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?
  echo "[$name] rc=$rc"
  case $rc in 0|1) return 0;; *) tail -20 $O/$name.err; exit $rc;; esac
}
bash tools/pmc_profile.sh $O/pmc "--steps 4 --warmup 2 --in-flight 1 --no-cpu-baseline --no-other-configs --no-viewpoints --no-full-mlp-leg" > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
python3 tools/mlp_traffic.py $O/pmc/summary.txt $O/point_mlp_traffic.json "round-6 final state" > /dev/null || exit 1
step trace 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 16 --warmup 3 --in-flight 1 --no-cpu-baseline --no-other-configs --no-viewpoints --no-full-mlp-leg
step shard 300 python tools/shard_balance.py --split gilv4096 --worlds 2,4,8 --reps 10 --in-flight 4
APN_DIST_BACKEND=gloo step gloo2 300 python bench.py --gpus 2 --steps 8 --warmup 2 --no-cpu-baseline --no-other-configs --no-viewpoints
find $O -name "*kernel_trace.csv" -delete; find $O -name "*counter_collection.csv" -delete
find $O -name "*_trace.csv" -size +4M -delete
du -sh $O; echo done
