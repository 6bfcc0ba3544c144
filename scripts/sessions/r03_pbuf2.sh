#!/bin/bash
# Path-buffer policies on one box: three buffers with compaction (copy) or without (DMT_PATH_COPY=0),
# two buffers (repair while minority <= 1/4; DMT_REPAIR_DIV=1: always), C3 and C5 draw + accept.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03pbuf2}
mkdir -p $O
K="python scripts/kbench.py --mapping lane --iters 20"
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread"
scripts/gpu_session.sh \
  "timeout -k 10 300 $PT tests/test_path_buffers.py > $O/pytest_pbuf.log 2>&1" \
  "timeout -k 10 150 $K --config c5 --accept > $O/c5_b3.json" \
  "DMT_PATH_COPY=0 timeout -k 10 150 $K --config c5 --accept > $O/c5_b3nc.json" \
  "DMT_PATH_BUFS=2 timeout -k 10 150 $K --config c5 --accept > $O/c5_b2.json" \
  "DMT_PATH_BUFS=2 DMT_REPAIR_DIV=1 timeout -k 10 150 $K --config c5 --accept > $O/c5_b2d1.json" \
  "timeout -k 10 150 $K --config c3 --accept > $O/c3_b3.json" \
  "DMT_PATH_COPY=0 timeout -k 10 150 $K --config c3 --accept > $O/c3_b3nc.json" \
  "DMT_PATH_BUFS=2 timeout -k 10 150 $K --config c3 --accept > $O/c3_b2.json" \
  "timeout -k 10 150 $K --config c3 --accept-all > $O/c3_accall.json" \
  "DMT_PATH_COPY=0 timeout -k 10 150 $K --config c5 --accept > $O/c5_b3nc_2.json" \
  "DMT_PATH_BUFS=2 timeout -k 10 150 $K --config c5 --accept > $O/c5_b2_2.json"
