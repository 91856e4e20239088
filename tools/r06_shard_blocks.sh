#!/bin/bash
# Shard of 8 (4 in flight) and the C2 line: early-termination MLP pass grid of 2048 workgroups
# (ab/mb2048) against the capacity-sized grid (ab/adapt: 512 for a shard of 8, 2048 for the frame).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
O=gpurun_out/r06sb; mkdir -p $O
for r in 1 2; do for b in ${VS:-mb2048 adapt}; do
  APN_HIP_LIB=$PWD/ab/$b/libapn_hip.so timeout -k 10 300 python tools/shard_balance.py --split gilv4096 --worlds 8 --reps 6 --in-flight 4 > $O/sb_${b}_$r.log 2>&1 || { tail -20 $O/sb_${b}_$r.log; exit 1; }
  grep -E "all shards re-timed" $O/sb_${b}_$r.log | sed "s/^/[$b] /"
done; done
[ -n "$SKIP_BENCH" ] && exit 0
BASE=mb2048 NEW=adapt SKIP_PARITY=1 SKIP_TAIL=1 bash tools/r06_mlp_ab.sh
