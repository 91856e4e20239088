source tools/gpu_steps.sh
step p1 300 bash tools/bench_rocprof.sh gpurun_out/prof_ax1
APN_HIP_LIB=ab/skwide/libapn_hip.so step p2 300 bash tools/bench_rocprof.sh gpurun_out/prof_ax2
python3 -c "
import csv
for d in ('gpurun_out/prof_ax1','gpurun_out/prof_ax2'):
  r=list(csv.DictReader(open(d+'/trace/run_kernel_stats.csv')))
  for x in r:
    if 'skeleton' in x['Name']: print(d, x['Calls'], float(x['AverageNs'])/1e3)
"
