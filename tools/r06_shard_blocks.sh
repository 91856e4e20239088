#!/bin/bash
# Shard of 8 (4 in flight): early-termination MLP pass grid of 512 / 1024 / 2048 workgroups (a
# shard's pass has ~1.8k tiles: at 2048 most workgroups run one tile after their weight staging).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
O=gpurun_out/r06sb; mkdir -p $O
for r in 1 2; do for b in 2048 512 1024; do
  APN_HIP_LIB=$PWD/ab/mb$b/libapn_hip.so timeout -k 10 300 python tools/shard_balance.py --split gilv4096 --worlds 8 --reps 6 --in-flight 4 > $O/sb_${b}_$r.log 2>&1 || { tail -20 $O/sb_${b}_$r.log; exit 1; }
  grep -E "all shards re-timed" $O/sb_${b}_$r.log | sed "s/^/[$b] /"
done; done
