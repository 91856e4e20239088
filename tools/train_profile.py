"""Profiling aid: torch.profiler view (ops grouped by input shapes) of the train_pcd step of
tools/train_bench.py, to attribute the GEMM kernels of the rocprof summary to their callers."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "articulated-point-nerf_amd")]
import torch  # noqa: E402
import train_bench as TB  # noqa: E402

sys.argv = [sys.argv[0], "--steps", "3", "--warmup", "2", "--no-cpu-baseline"] + sys.argv[1:]
from torch.profiler import profile, ProfilerActivity  # noqa: E402

with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    TB.main()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=30,
                                                         max_name_column_width=40, max_shapes_column_width=70))
