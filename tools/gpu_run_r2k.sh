source tools/gpu_steps.sh
export AB_STEPS=10
step tests 150 python -u -m pytest tests/test_mlp_precision.py tests/test_hip_parity.py -m gpu -q -x -rf --timeout 100 --timeout-method thread -k "mlp or precision or same_cloud or golden" > gpurun_out/gpu_tests12.log 2>&1
tail -2 gpurun_out/gpu_tests12.log
step ab 900 bash tools/ab.sh "APN_AB=cur" "APN_AB=cur2"
step bench_r1 300 bash -c 'cd ab/r1 && python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > ../../gpurun_out/bench12_r1.json 2> ../../gpurun_out/bench12_r1.err'
python3 -c "import json; d=json.load(open('gpurun_out/bench12_r1.json')); print('r1', d['ms_per_step'], d['stage_ms'])"
