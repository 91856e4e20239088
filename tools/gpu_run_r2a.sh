set -o pipefail
mkdir -p gpurun_out
echo "== debug band"; timeout -k 10 300 python -u tools/debug_band.py C3 rgb_marched_direct > gpurun_out/debug_band.log 2>&1; echo "rc=$?"
echo "== tests"; timeout -k 10 600 python -u -m pytest tests/test_0_shard_spawn.py tests/test_mlp_precision.py tests/test_hip_parity.py -m gpu -q -rf --timeout 300 --timeout-method thread -k "spawn or precision or sticky or band or same_cloud or golden_same or mlp_stage" > gpurun_out/gpu_tests2.log 2>&1; echo "rc=$?"
echo "== bench"; timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench2.json 2> gpurun_out/bench2.err; echo "rc=$?"
echo "== gloo 2-rank shard rehearsal"; APN_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err; echo "rc=$?"
echo "== gloo 2-rank C5"; APN_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config C5 --steps 10 --warmup 2 > gpurun_out/bench_gloo2_c5.json 2> gpurun_out/bench_gloo2_c5.err; echo "rc=$?"
tail -5 gpurun_out/gpu_tests2.log; cat gpurun_out/bench2.json gpurun_out/bench_gloo2.json gpurun_out/bench_gloo2_c5.json
