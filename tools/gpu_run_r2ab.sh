source tools/gpu_steps.sh
step tests 900 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_ab.log 2>&1
tail -3 gpurun_out/gpu_tests_ab.log
AB_STEPS=20 step ab 600 bash tools/ab.sh "APN_AB=new" "APN_INBBOX_FILL=ray" "APN_AB=new2"
step rocprof 400 bash tools/bench_rocprof.sh gpurun_out/prof_ab
python3 -c "
import csv
r=list(csv.DictReader(open('gpurun_out/prof_ab/trace/run_kernel_stats.csv')))
for x in r[:16]: print(x['Name'][:60], x['Calls'], '%.4f'%(float(x['AverageNs'])/1e6))
"
