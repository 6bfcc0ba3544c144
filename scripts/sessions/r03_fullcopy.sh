#!/bin/bash
# Consolidation writing whole lines (DMT_FULL_COPY=1: the majority lanes rewrite their own u
# beside the copied lanes) vs the default (only the lanes outside the majority's buffer copy),
# C5 and C3 draw + accept loops on one box, interleaved; path-buffer parity tests first.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03fc}
mkdir -p $O
K="python scripts/kbench.py --mapping lane --iters 20"
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread"
scripts/gpu_session.sh \
  "timeout -k 10 300 $PT tests/test_path_buffers.py > $O/pytest_pbuf.log 2>&1" \
  "timeout -k 10 150 $K --config c5 --accept > $O/c5_def1.json" \
  "DMT_FULL_COPY=1 timeout -k 10 150 $K --config c5 --accept > $O/c5_full1.json" \
  "timeout -k 10 150 $K --config c5 --accept > $O/c5_def2.json" \
  "DMT_FULL_COPY=1 timeout -k 10 150 $K --config c5 --accept > $O/c5_full2.json" \
  "timeout -k 10 150 $K --config c3 --accept > $O/c3_def1.json" \
  "DMT_FULL_COPY=1 timeout -k 10 150 $K --config c3 --accept > $O/c3_full1.json"
