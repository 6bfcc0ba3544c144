#!/bin/bash
# Last check of the session's final tree: GPU suite and smoke.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zy
mkdir -p $O
scripts/gpu_session.sh \
 "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1" \
 "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1"
