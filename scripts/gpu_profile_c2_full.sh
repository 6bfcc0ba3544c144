#!/bin/bash
# Full C2 profile: bench line (with CPU baseline), rocprofv3 kernel trace (warmup = steps, so
# every dispatch of the persistent kernel runs the same 500 iterations and the trace's average
# duration is the bench's kernel_avg_us), PMC FETCH/WRITE passes
# (10 iterations per dispatch), calibration, SQ issue/wait passes.  usage: <outdir-name>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64"
B="python bench.py --steps 10 --warmup 10 --no-cpu-baseline"
scripts/gpu_session.sh \
 "timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python bench.py --steps 500 --warmup 500 --no-cpu-baseline > $O/prof_c2.log 2>&1" \
 "timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_c2_fetch -o f --output-format csv -- $B > $O/pmc_c2_fetch.log 2>&1" \
 "timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c2_write -o w --output-format csv -- $B > $O/pmc_c2_write.log 2>&1" \
 "timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_calib_fetch -o f --output-format csv -- scripts/calib_stream > $O/calib_f.log 2>&1" \
 "timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_calib_write -o w --output-format csv -- scripts/calib_stream > $O/calib_w.log 2>&1" \
 "timeout -s KILL 120 rocprofv3 --pmc $P1 -d $O/sq_p1 -o p --output-format csv -- $B > $O/sq_p1.log 2>&1" \
 "timeout -s KILL 120 rocprofv3 --pmc $P2 -d $O/sq_p2 -o p --output-format csv -- $B > $O/sq_p2.log 2>&1" \
 "timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 20 --warmup 3 > $O/bench_c3.json 2> $O/bench_c3.err" \
 "timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 20 --warmup 3 > $O/bench_c5.json 2> $O/bench_c5.err"
