source tools/gpu_steps.sh
step bench_c5 300 python -u bench.py --config C5 --steps 60 --warmup 5 -o gpurun_out/bench23_c5.json
python3 -c "
import json; d=json.load(open('gpurun_out/bench23_c5.json')); print(d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['cpu_baseline'])"
