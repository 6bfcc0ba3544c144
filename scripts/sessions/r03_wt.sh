#!/bin/bash
# r02zi follow-up: the GPU suite on a write-through (sc1) path-store build.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03x}
mkdir -p $O
scripts/gpu_session.sh \
  "DMT_LIB_PATH=build_variants/wt/libdmt.so timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_wt.log 2>&1"
