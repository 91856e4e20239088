source tools/gpu_steps.sh
step frame_graph_tests 300 python -u -m pytest tests/test_frame_graph.py -x -v --timeout 120 --timeout-method thread
step bench_c2_default 600 python -u bench.py -o gpurun_out/r2z_c2.json
