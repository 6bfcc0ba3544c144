#!/bin/bash
# Three path buffers per container (MAP_LANE): the new parity tests, the whole GPU suite, then
# C3/C5 draw time in a draw + accept loop with three buffers and with two (DMT_PATH_BUFS=2).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03pbuf}
mkdir -p $O
K="python scripts/kbench.py --mapping lane --iters 20"
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread"
scripts/gpu_session.sh \
  "timeout -k 10 300 $PT tests/test_path_buffers.py > $O/pytest_pbuf.log 2>&1" \
  "timeout -k 10 800 $PT tests -m gpu > $O/pytest_gpu.log 2>&1" \
  "timeout -k 10 150 $K --config c3 --accept > $O/c3acc_b3.json" \
  "DMT_PATH_BUFS=2 timeout -k 10 150 $K --config c3 --accept > $O/c3acc_b2.json" \
  "timeout -k 10 150 $K --config c5 --accept > $O/c5acc_b3.json" \
  "DMT_PATH_BUFS=2 timeout -k 10 150 $K --config c5 --accept > $O/c5acc_b2.json" \
  "timeout -k 10 150 $K --config c3 --accept > $O/c3acc_b3b.json" \
  "timeout -k 10 150 $K --config c5 --accept > $O/c5acc_b3b.json"
