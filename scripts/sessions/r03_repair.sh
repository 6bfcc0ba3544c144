#!/bin/bash
# C3/C5 draw time inside a draw + accept loop (scripts/kbench.py --accept) by tile-phase repair
# threshold (DMT_REPAIR_DIV: repair while minority <= active/div; 64: at most one lane;
# 1000000: never) and minimum minority (DMT_REPAIR_MIN), against draw-only (uniform selectors) and accept-all loops.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03rep}
mkdir -p $O
K="python scripts/kbench.py --mapping lane --iters 20"
scripts/gpu_session.sh \
  "timeout -k 10 150 $K --config c3 --accept > $O/c3acc_div4.json" \
  "DMT_REPAIR_DIV=64 timeout -k 10 150 $K --config c3 --accept > $O/c3acc_div64.json" \
  "DMT_REPAIR_DIV=1000000 timeout -k 10 150 $K --config c3 --accept > $O/c3acc_never.json" \
  "timeout -k 10 150 $K --config c3 --accept-all > $O/c3accall.json" \
  "timeout -k 10 150 $K --config c3 > $O/c3draw.json" \
  "DMT_REPAIR_MIN=4 timeout -k 10 150 $K --config c3 --accept > $O/c3acc_min4.json" \
  "DMT_REPAIR_MIN=8 timeout -k 10 150 $K --config c3 --accept > $O/c3acc_min8.json" \
  "DMT_REPAIR_MIN=16 timeout -k 10 150 $K --config c3 --accept > $O/c3acc_min16.json" \
  "timeout -k 10 150 $K --config c3 --accept > $O/c3acc_div4b.json" \
  "DMT_REPAIR_DIV=1 timeout -k 10 150 $K --config c5 --accept > $O/c5acc_div1.json" \
  "timeout -k 10 150 $K --config c5 --accept > $O/c5acc_div4.json"
