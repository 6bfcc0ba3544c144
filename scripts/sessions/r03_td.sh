#!/bin/bash
# Time-dependent auxiliary laws: their GPU parity tests, then the whole GPU suite.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03y}
mkdir -p $O
scripts/gpu_session.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_td_aux.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_td.log 2>&1" \
  "timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1"
