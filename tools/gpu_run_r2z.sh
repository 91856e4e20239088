#!/bin/bash
# Kernel stats of one rank's frame of the 8-way blocks split, and of the full frame.
source tools/gpu_steps.sh
step sp8b 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sp8b -o sp8b --output-format csv -- python3 tools/shard_profile.py --world 8 > gpurun_out/sp8b.log 2>&1
