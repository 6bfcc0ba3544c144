#!/bin/bash
# C5 producer/consumer split (DMT_LANE_SPLIT=1) vs single wave: SQ issue counters per kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zb
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
NB="--no-cpu-baseline --steps 3 --warmup 1"
scripts/gpu_session.sh \
 "DMT_LANE_SPLIT=1 timeout -s KILL 200 rocprofv3 --pmc $P1 -d $O/ps_sq1 -o p --output-format csv -- python bench.py --config c5 $NB > $O/ps_sq1.log 2>&1" \
 "timeout -s KILL 200 rocprofv3 --pmc $P1 -d $O/k_sq1 -o p --output-format csv -- python bench.py --config c5 $NB > $O/k_sq1.log 2>&1"
