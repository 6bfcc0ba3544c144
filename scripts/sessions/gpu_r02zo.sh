#!/bin/bash
# Host-side breakdown of one dmt_mcmc_run call (DMT_HOST_PROFILE): pre-launch, launch API, wait.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zo
mkdir -p $O
scripts/gpu_session.sh \
 "DMT_HOST_PROFILE=1 timeout -k 10 120 python scripts/first_call_probe.py > $O/fc.json 2> $O/fc.err" \
 "DMT_HOST_PROFILE=1 DMT_DISPATCH_EVENTS=0 timeout -k 10 120 python scripts/first_call_probe.py > $O/fc_rec.json 2> $O/fc_rec.err" \
 "DMT_HOST_PROFILE=1 DMT_SPIN_WAIT=0 timeout -k 10 120 python scripts/first_call_probe.py > $O/fc_block.json 2> $O/fc_block.err"
