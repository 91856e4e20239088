source tools/gpu_steps.sh
t() { python -u -m pytest tests/test_0_shard_spawn.py -q -x --timeout 200 --timeout-method thread 2>&1 | grep -E "passed|failed|AssertionError: frame" | head -3; }
echo "== current"; t
echo "== composite seq"; APN_COMPOSITE=seq t
echo "== no bpf1"; APN_HIP_LIB=ab/nobpf/libapn_hip.so t
echo "== no bpf1 + seq"; APN_COMPOSITE=seq APN_HIP_LIB=ab/nobpf/libapn_hip.so t
