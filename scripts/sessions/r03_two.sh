#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03two}
mkdir -p $O
scripts/gpu_session.sh \
  "DMT_SVC_STATS=1 timeout -k 10 300 python -u -m pytest tests/test_deferred.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1"
