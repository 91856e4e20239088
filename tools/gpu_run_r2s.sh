source tools/gpu_steps.sh
step bench 300 python -u bench.py --steps 20 --warmup 3 -o gpurun_out/bench20.json
python3 -c "
import json
d=json.load(open('gpurun_out/bench20.json')); print(d['value']/1e6, d['ms_per_step'], d['config']['step'], d['stage_ms'], d['cpu_baseline'], d.get('same_cloud_vs_oracle'))"
step ab_c5 300 bash tools/ab_c5.sh "APN_AB=cur" "APN_HIP_LIB=ab/nt/libapn_hip.so"
