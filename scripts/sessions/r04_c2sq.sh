#!/bin/bash
# Round 4, last tree: C2 SQ issue passes and PMC FETCH/WRITE passes of k_mcmc_resident_pc.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04c2sq}
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64"
B2="python bench.py --steps 20 --warmup 20 --no-cpu-baseline --repeats 0 --calls-iters 0"
scripts/gpu_session.sh \
 "timeout -s KILL 120 rocprofv3 --pmc $P1 -d $O/c2_sq1 -o p --output-format csv -- $B2 > $O/c2_sq1.log 2>&1" \
 "timeout -s KILL 120 rocprofv3 --pmc $P2 -d $O/c2_sq2 -o p --output-format csv -- $B2 > $O/c2_sq2.log 2>&1" \
 "timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_c2_fetch -o f --output-format csv -- $B2 > $O/pmc_c2_fetch.log 2>&1" \
 "timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c2_write -o w --output-format csv -- $B2 > $O/pmc_c2_write.log 2>&1"
