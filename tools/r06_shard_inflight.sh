#!/bin/bash
# Ray shards of 2 / 4 / 8 with 3 and 4 frames in flight (same box): does a deeper pipeline hide
# the short launches' latency tails (kNN passes, replicated stages)?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
O=gpurun_out/r06s; mkdir -p $O
for n in ${NS:-3 4}; do
  timeout -k 10 300 python tools/shard_balance.py --split gilv4096 --worlds ${WORLDS:-8} --reps 6 --in-flight $n > $O/sb_$n.log 2>&1 || { tail -20 $O/sb_$n.log; exit 1; }
  grep -E "all shards re-timed" $O/sb_$n.log | sed "s/^/[$n] /"
done
