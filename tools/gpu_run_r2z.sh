#!/bin/bash
# Kernel stats of one rank's frame of the 8-way blocks split, and of the full frame.
source tools/gpu_steps.sh
step sp8 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sp8 -o sp8 --output-format csv -- python3 tools/shard_profile.py --world 8 > gpurun_out/sp8.log 2>&1
step sp1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sp1 -o sp1 --output-format csv -- python3 tools/shard_profile.py --world 1 > gpurun_out/sp1.log 2>&1
