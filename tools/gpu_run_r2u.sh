source tools/gpu_steps.sh
step bench 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline -o gpurun_out/bench22.json 2> gpurun_out/bench22.err
grep -h "host time\|stage ms" gpurun_out/bench22.err
step ab_c5 300 bash tools/ab_c5.sh "APN_AB=cur" "APN_HIP_LIB=ab/nt/libapn_hip.so"
step pmc 900 bash tools/pmc_profile.sh gpurun_out/r02_pmc --steps 2 --warmup 1 --no-cpu-baseline
python3 -c "
import json; d=json.load(open('gpurun_out/r02_pmc/summary.txt'))
for k in list(d)[:4]: print(k, {a: (round(b,4) if isinstance(b,float) else b) for a,b in d[k].items()})"
