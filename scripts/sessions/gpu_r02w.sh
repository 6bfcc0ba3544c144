#!/bin/bash
# Round 2: GPU suite after recompute_path skip, snapshots inside mcmc_run, PC kernel template.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02w
mkdir -p $O
scripts/gpu_session.sh \
 "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1"
