source tools/gpu_steps.sh
t() { python -u -m pytest tests/test_0_shard_spawn.py -q -x --timeout 200 --timeout-method thread 2>&1 | grep -E "passed|failed|AssertionError: frame" | head -2; }
for k in 1 2 3 4 5 6; do echo "== spill-free $k"; t; done
