#!/bin/bash
# Round 2: host wait strategies (polling vs blocking, spin scheduling) on the driver's command.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02j
mkdir -p $O
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
scripts/gpu_session.sh \
 "timeout -k 10 300 $B > $O/poll.json 2> $O/poll.err" \
 "DMT_SPIN_WAIT=0 timeout -k 10 300 $B > $O/block.json 2> $O/block.err" \
 "DMT_SPIN_WAIT=0 DMT_SYNC_SPIN=1 timeout -k 10 300 $B > $O/block_spinflag.json 2> $O/block_spinflag.err" \
 "DMT_SYNC_SPIN=1 timeout -k 10 300 $B > $O/poll_spinflag.json 2> $O/poll_spinflag.err" \
 "timeout -k 10 300 $B > $O/poll2.json 2> $O/poll2.err" \
 "DMT_SPIN_WAIT=0 timeout -k 10 300 $B > $O/block2.json 2> $O/block2.err" \
 "timeout -k 10 200 python scripts/runbench.py > $O/run_poll.json 2> $O/run_poll.err"
