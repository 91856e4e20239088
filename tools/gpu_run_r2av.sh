source tools/gpu_steps.sh
step tests 600 python -u -m pytest tests/test_hip_parity.py tests/test_frame_graph.py -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_av.log 2>&1
tail -1 gpurun_out/gpu_tests_av.log
step rocprof 400 bash tools/bench_rocprof.sh gpurun_out/prof_av
python3 -c "
import csv, json
r=list(csv.DictReader(open('gpurun_out/prof_av/trace/run_kernel_stats.csv')))
for x in r:
  if 'coarse' in x['Name'] or 'sum27' in x['Name']: print(x['Name'][:50], x['Calls'], float(x['AverageNs'])/1e3)
b=json.load(open('gpurun_out/prof_av/bench.json')); print(b['value']/1e6, b['ms_per_step'], b['stage_ms'])
"
