source tools/gpu_steps.sh
step probe 300 python -u tools/determinism_probe.py 25
APN_CONCURRENT_GRID=0 step probe_serial 300 python -u tools/determinism_probe.py 25 | tail -3
