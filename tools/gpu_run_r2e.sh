source tools/gpu_steps.sh
step tests 600 python -u -m pytest tests/test_lbs_paths.py tests/test_hip_parity.py -m gpu -q -rf --timeout 300 --timeout-method thread -k "lbs or repose or skeleton or pointwarper or records or sampling or forward_vs" > gpurun_out/gpu_tests6.log 2>&1
tail -3 gpurun_out/gpu_tests6.log
step bench_c5 300 python -u bench.py --config C5 --steps 60 --warmup 5 --no-cpu-baseline -o gpurun_out/bench6_c5.json
cat gpurun_out/bench6_c5.json
step ab 900 bash tools/ab.sh "APN_AB=cur" "APN_HIP_LIB=ab/noguard/libapn_hip.so" "APN_KNN_SUBDIV=6" "APN_KNN_SUBDIV=4" "APN_KNN_SUBDIV=10"
step bench_r1 300 bash -c 'cd ab/r1 && python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > ../../gpurun_out/bench6_r1.json 2> ../../gpurun_out/bench6_r1.err'
python3 -c "import json; d=json.load(open('gpurun_out/bench6_r1.json')); print('r1', d['ms_per_step'], d['stage_ms'])"
