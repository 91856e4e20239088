#!/bin/bash
# Measured once (round 5) with an APN_DIRECT_SIDE switch in temporalpoints.py, since removed: the
# direct-blend kernel on the grid's side stream beside the MLP passes vs inside apn_point_mlp_ert,
# 3 and 4 frames in flight. Side stream: 6.58-6.60 ms/frame at 3 in flight (no overlap left) vs
# 5.91-5.95 inside; 4 in flight 5.95-5.99 either way. Kept as the record of the A/B loop.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do for ds in 0 1; do for n in 3 4; do
APN_DIRECT_SIDE=$ds timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --in-flight $n --no-cpu-baseline --no-other-configs --no-full-mlp-leg --no-viewpoints -o gpurun_out/ab_side_${ds}_${n}.json > /dev/null 2>&1 || exit 1
python -c "import json; d=json.load(open('gpurun_out/ab_side_${ds}_${n}.json')); print('side=$ds n=$n', round(d['ms_per_step'],3), 'serial', round(d['config']['serial_ms_per_step'],3))"
done; done; done
