source tools/gpu_steps.sh
step tests 900 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests19.log 2>&1
tail -3 gpurun_out/gpu_tests19.log
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline -o gpurun_out/bench19.json
step bench_eager 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --graph off -o gpurun_out/bench19_eager.json
python3 -c "
import json
for f in ('gpurun_out/bench19.json','gpurun_out/bench19_eager.json'):
    d=json.load(open(f)); print(f, d['value']/1e6, d['ms_per_step'], d['config']['step'], d['stage_ms'])"
step ab_c5 300 bash tools/ab_c5.sh "APN_AB=cur" "APN_HIP_LIB=ab/nt/libapn_hip.so"
