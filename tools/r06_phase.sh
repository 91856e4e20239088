#!/bin/bash
# Per-phase cycle split of the 128-row MLP kernel (debug library, APN_MLP_VARIANT=5: clock64 per phase
# on wave 0 of every workgroup). The timed kernel is the non-listed one, which the bench's full-MLP
# leg (early ray termination off) runs; the early-termination passes run the untimed listed kernel.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
O=gpurun_out/r06p; mkdir -p $O
APN_HIP_LIB=${LIB:-$PWD/articulated-point-nerf_amd/apn_amd/libapn_hip_debug.so} APN_MLP_VARIANT=5 timeout -k 10 300 \
  python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-other-configs --no-viewpoints -o $O/phase${TAG}.json \
  2> $O/phase${TAG}.err > /dev/null || { tail -20 $O/phase${TAG}.err; exit 1; }
grep -E "mlp phases|full MLP" $O/phase${TAG}.err
