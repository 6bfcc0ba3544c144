#!/bin/bash
# Adaptive path buffers (path_plan): parity tests, the GPU suite, then C3/C5 draw + accept times
# by policy on one box (default; two buffers; two buffers with the old repair threshold 4).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03pbuf3}
mkdir -p $O
K="python scripts/kbench.py --mapping lane --iters 20"
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread"
scripts/gpu_session.sh \
  "timeout -k 10 300 $PT tests/test_path_buffers.py > $O/pytest_pbuf.log 2>&1" \
  "timeout -k 10 150 $K --config c3 --accept > $O/c3_def.json" \
  "timeout -k 10 150 $K --config c5 --accept > $O/c5_def.json" \
  "DMT_PATH_BUFS=2 DMT_REPAIR_DIV=4 timeout -k 10 150 $K --config c3 --accept > $O/c3_old.json" \
  "DMT_PATH_BUFS=2 DMT_REPAIR_DIV=4 timeout -k 10 150 $K --config c5 --accept > $O/c5_old.json" \
  "timeout -k 10 150 $K --config c3 --accept > $O/c3_def2.json" \
  "timeout -k 10 150 $K --config c5 --accept > $O/c5_def2.json" \
  "timeout -k 10 800 $PT tests -m gpu > $O/pytest_gpu.log 2>&1"
