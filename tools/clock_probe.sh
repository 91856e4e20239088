#!/bin/bash
# Per-kernel shader clock of an A/B variant: one rocprofv3 pass (kernel trace + GRBM_GUI_ACTIVE,
# SQ_BUSY_CYCLES, SQ_VALU_MFMA_BUSY_CYCLES) over a short bench run with APN_HIP_LIB=ab/<tag>.
# Usage on the GPU box: VARIANTS="base m32" bash tools/clock_probe.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in $VARIANTS; do
  OUT=gpurun_out/clk_$v; rm -rf $OUT; mkdir -p $OUT
  APN_HIP_LIB=$PWD/ab/$v/libapn_hip.so timeout -k 10 200 rocprofv3 --kernel-trace \
    --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES -d $OUT -o run --output-format csv \
    -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-other-configs > $OUT/b.json 2> $OUT/b.err || exit 1
  python3 tools/clock_summary.py $OUT "$v" || exit 1
  find $OUT -name "*.csv" -size +1M -delete
done
