source tools/gpu_steps.sh
step tests 900 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_t.log 2>&1
tail -3 gpurun_out/gpu_tests_t.log
AB_STEPS=20 step ab 600 bash tools/ab.sh "APN_AB=merged" "APN_KNN_B_SPLIT=1" "APN_AB=merged2" "APN_KNN_B_SPLIT=1"
step rocprof 400 bash tools/bench_rocprof.sh gpurun_out/prof_t
python3 -c "
import csv
r=list(csv.DictReader(open('gpurun_out/prof_t/trace/run_kernel_stats.csv')))
for x in r[:12]: print(x['Name'][:60], x['Calls'], '%.4f'%(float(x['AverageNs'])/1e6))
"
