source tools/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step trprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trprof -o run --output-format csv -- python3 tools/train_bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/trprof.json 2> gpurun_out/trprof.err
cat gpurun_out/trprof.json
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/trprof/**/*kernel_stats.csv', recursive=True)[0]
r = list(csv.DictReader(open(f)))
tot = sum(float(x['TotalDurationNs']) for x in r) / 1e6
calls = sum(int(x['Calls']) for x in r)
print(f"kernels: {calls} launches, {tot:.2f} ms total over 13 steps -> {tot/13:.2f} ms/step, {calls/13:.0f} launches/step")
for x in r[:25]:
    print('%-80s %5d %8.3f' % (x['Name'][:80], int(x['Calls']), float(x['TotalDurationNs'])/1e6/13))
PY
