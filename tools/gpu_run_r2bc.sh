source tools/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bc -o run --output-format csv -- python3 tools/shard_balance.py --split cost --worlds 8 --reps 5 > gpurun_out/bal_bc.log 2>&1
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/prof_bc/**/*kernel_stats.csv', recursive=True)[0]
r = list(csv.DictReader(open(f)))
for x in r[:22]:
    print('%-60s %6d avg %8.1f us' % (x['Name'][:60], int(x['Calls']), float(x['AverageNs'])/1e3))
PY
