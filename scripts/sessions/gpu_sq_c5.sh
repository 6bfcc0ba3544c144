#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F32"
P3="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"
B="python bench.py --config ${2:-c5} --steps 3 --warmup 1 --no-cpu-baseline"
scripts/gpu_session.sh \
 "timeout -s KILL 150 rocprofv3 --pmc $P1 -d $O/p1 -o p --output-format csv -- $B > $O/p1.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc $P2 -d $O/p2 -o p --output-format csv -- $B > $O/p2.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc $P3 -d $O/p3 -o p --output-format csv -- $B > $O/p3.log 2>&1"
