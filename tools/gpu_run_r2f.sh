source tools/gpu_steps.sh
step tests 900 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests7.log 2>&1
tail -3 gpurun_out/gpu_tests7.log
step ab 600 bash tools/ab.sh "APN_AB=cur" "APN_AB=cur2"
step bench_r1 300 bash -c 'cd ab/r1 && python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > ../../gpurun_out/bench7_r1.json 2> ../../gpurun_out/bench7_r1.err'
python3 -c "import json; d=json.load(open('gpurun_out/bench7_r1.json')); print('r1', d['ms_per_step'], d['stage_ms'])"
