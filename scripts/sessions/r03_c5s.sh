#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03c5s}
mkdir -p $O
scripts/gpu_session.sh \
  "timeout -k 10 400 python -u scripts/c5_scaling.py 16384 32768 65536 > $O/c5_scaling.log 2>&1"
