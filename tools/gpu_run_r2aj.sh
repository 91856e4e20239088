source tools/gpu_steps.sh
t() { python -u -m pytest tests/test_0_shard_spawn.py -q -x --timeout 200 --timeout-method thread 2>&1 | grep -E "passed|failed|AssertionError: frame" | head -2; }
for k in 1 2 3; do echo "== default $k"; t; done
for k in 1 2 3; do echo "== serial grid $k"; APN_CONCURRENT_GRID=0 t; done
for k in 1 2 3; do echo "== nobpf $k"; APN_HIP_LIB=ab/nobpf/libapn_hip.so t; done
