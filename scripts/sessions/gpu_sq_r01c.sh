#!/bin/bash
# SQ/GRBM counter passes (issue vs wait breakdown) of the C2 persistent kernel and the C3 lane
# kernel; each pass its own run (rocprofv3 does not split counters over passes).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r01c_sq
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH"
scripts/gpu_session.sh \
 "timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1" \
 "timeout -s KILL 120 rocprofv3 --pmc $P1 -d $O/c2_p1 -o p --output-format csv -- python bench.py --steps 10 --warmup 10 --no-cpu-baseline > $O/c2_p1.log 2>&1" \
 "timeout -s KILL 120 rocprofv3 --pmc $P2 -d $O/c2_p2 -o p --output-format csv -- python bench.py --steps 10 --warmup 10 --no-cpu-baseline > $O/c2_p2.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc $P1 -d $O/c3_p1 -o p --output-format csv -- python bench.py --config c3 --steps 4 --warmup 2 --no-cpu-baseline > $O/c3_p1.log 2>&1"
