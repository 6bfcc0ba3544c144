#!/bin/bash
# C2 through the per-iteration kernels (the path a draw_proposal_path!/accept_reject_proposal_path!
# caller takes): bench line and SQ counters of k_block_scan.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
export DMT_MCMC_PERSIST=0
scripts/gpu_session.sh \
 "timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 > $O/c2_step.json 2> $O/c2_step.err" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o c2 --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1" \
 "timeout -s KILL 120 rocprofv3 --pmc $P1 -d $O/sq -o p --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/sq.log 2>&1"
