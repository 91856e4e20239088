source tools/gpu_steps.sh
step tests 600 python -u -m pytest tests/test_hip_parity.py tests/test_frame_graph.py tests/test_0_shard_spawn.py -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_ay.log 2>&1
tail -1 gpurun_out/gpu_tests_ay.log
AB_STEPS=20 step ab 600 bash tools/ab.sh "APN_AB=tiled" "APN_CELL_BOUND=cell" "APN_AB=tiled2" "APN_CELL_BOUND=cell"
step rocprof 400 bash tools/bench_rocprof.sh gpurun_out/prof_ay
python3 -c "
import csv
r=list(csv.DictReader(open('gpurun_out/prof_ay/trace/run_kernel_stats.csv')))
for x in r:
  if 'cell_bound' in x['Name'] or 'tile_list' in x['Name'] or 'mark_cells' in x['Name']: print(x['Name'][:50], x['Calls'], float(x['AverageNs'])/1e3)
"
