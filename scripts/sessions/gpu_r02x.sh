#!/bin/bash
# Round 2 evidence for C3 / C5 on the current build: bench lines with the CPU legs, rocprofv3
# kernel traces, FETCH/WRITE PMC passes (+ calibration), SQ passes of the C5 draw kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02x
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F32"
NB="--no-cpu-baseline"
scripts/gpu_session.sh \
 "timeout -k 10 400 python bench.py --config c3 --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err" \
 "timeout -k 10 400 python bench.py --config c5 --steps 20 --warmup 5 > $O/bench_c5.json 2> $O/bench_c5.err" \
 "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o c3 --output-format csv -- python bench.py --config c3 --steps 20 --warmup 5 $NB > $O/prof_c3.log 2>&1" \
 "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o c5 --output-format csv -- python bench.py --config c5 --steps 20 --warmup 5 $NB > $O/prof_c5.log 2>&1" \
 "timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_c3_fetch -o f --output-format csv -- python bench.py --config c3 --steps 4 --warmup 1 $NB > $O/pmc_c3_fetch.log 2>&1" \
 "timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c3_write -o w --output-format csv -- python bench.py --config c3 --steps 4 --warmup 1 $NB > $O/pmc_c3_write.log 2>&1" \
 "timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_c5_fetch -o f --output-format csv -- python bench.py --config c5 --steps 4 --warmup 1 $NB > $O/pmc_c5_fetch.log 2>&1" \
 "timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c5_write -o w --output-format csv -- python bench.py --config c5 --steps 4 --warmup 1 $NB > $O/pmc_c5_write.log 2>&1" \
 "timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_calib_fetch -o f --output-format csv -- scripts/calib_stream > $O/calib_f.log 2>&1" \
 "timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_calib_write -o w --output-format csv -- scripts/calib_stream > $O/calib_w.log 2>&1" \
 "timeout -s KILL 200 rocprofv3 --pmc $P1 -d $O/c5_sq1 -o p --output-format csv -- python bench.py --config c5 --steps 4 --warmup 1 $NB > $O/c5_sq1.log 2>&1" \
 "timeout -s KILL 200 rocprofv3 --pmc $P2 -d $O/c5_sq2 -o p --output-format csv -- python bench.py --config c5 --steps 4 --warmup 1 $NB > $O/c5_sq2.log 2>&1" \
 "timeout -s KILL 200 rocprofv3 --pmc $P1 -d $O/c3_sq1 -o p --output-format csv -- python bench.py --config c3 --steps 4 --warmup 1 $NB > $O/c3_sq1.log 2>&1"
