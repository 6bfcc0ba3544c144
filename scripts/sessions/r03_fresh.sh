#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03fresh}
mkdir -p $O
scripts/gpu_session.sh \
  "timeout -k 10 120 python -u scripts/ou_fresh_check.py > $O/fresh.log 2>&1" \
  "timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1" \
  "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1"
