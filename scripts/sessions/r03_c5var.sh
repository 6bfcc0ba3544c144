#!/bin/bash
# C5 draw + accept on the path-buffer build: single-lane kernel (default) vs the producer/consumer
# split (DMT_LANE_SPLIT=1) vs lane pairs (DMT_LANE_PAIR=1), interleaved on one box.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03c5v}
mkdir -p $O
K="python scripts/kbench.py --mapping lane --iters 20 --config c5 --accept"
scripts/gpu_session.sh \
  "DMT_LANE_SPLIT=0 timeout -k 10 150 $K > $O/def1.json" \
  "DMT_LANE_SPLIT=1 timeout -k 10 150 $K > $O/split1.json" \
  "DMT_LANE_SPLIT=0 DMT_LANE_PAIR=1 timeout -k 10 150 $K > $O/pair1.json" \
  "DMT_LANE_SPLIT=0 timeout -k 10 150 $K > $O/def2.json" \
  "DMT_LANE_SPLIT=1 timeout -k 10 150 $K > $O/split2.json" \
  "DMT_LANE_SPLIT=0 DMT_LANE_PAIR=1 timeout -k 10 150 $K > $O/pair2.json"
