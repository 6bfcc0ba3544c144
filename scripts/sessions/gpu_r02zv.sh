#!/bin/bash
# C3 on the final build: PMC traffic (FETCH/WRITE + stream calibration) and SQ issue counters of
# the lane kernel (k_block, FHN fp64), for profiles/r02zv_traffic_c3.json / r02zv_issue_c3.json.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zv
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64"
B="python bench.py --config c3 --steps 4 --warmup 2 --no-cpu-baseline"
scripts/gpu_session.sh \
 "timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_c3_fetch -o f --output-format csv -- $B > $O/pmc_c3_fetch.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c3_write -o w --output-format csv -- $B > $O/pmc_c3_write.log 2>&1" \
 "timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_calib_fetch -o f --output-format csv -- scripts/calib_stream > $O/calib_f.log 2>&1" \
 "timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_calib_write -o w --output-format csv -- scripts/calib_stream > $O/calib_w.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc $P1 -d $O/c3_sq1 -o p --output-format csv -- $B > $O/c3_sq1.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc $P2 -d $O/c3_sq2 -o p --output-format csv -- $B > $O/c3_sq2.log 2>&1"
