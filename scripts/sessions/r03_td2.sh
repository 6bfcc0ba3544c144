#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03z}
mkdir -p $O
scripts/gpu_session.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_td_aux.py tests/test_reference_tutorials.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_td.log 2>&1"
