#!/bin/bash
# Round 4: SQ issue passes of the lane draw kernels on the shipped tree (C5 packets, C3 rows),
# C3 rocprofv3 kernel stats and PMC passes, C5 rolling-prefetch A/B.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04d}
mkdir -p $O
K="python scripts/kbench.py --mapping lane"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64"
B5="python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline --calls-iters 0 --repeats 0"
B3="python bench.py --config c3 --steps 4 --warmup 2 --no-cpu-baseline --calls-iters 0 --repeats 0"
P=scripts/c5_layout_probe
scripts/gpu_session.sh \
 "timeout -k 10 90 $P 512 10 pk > $O/probe.jsonl 2> $O/probe.err" \
 "timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_pfetch -o f --output-format csv -- $P 512 2 pk > $O/pmc_pfetch.log 2>&1" \
 "timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_pwrite -o w --output-format csv -- $P 512 2 pk > $O/pmc_pwrite.log 2>&1" \
 "timeout -k 10 150 $K --config c5 --accept > $O/c5_roll.json 2> $O/c5_roll.err" \
 "DMT_LIB_PATH=build_variants/libdmt_noroll.so timeout -k 10 150 $K --config c5 --accept > $O/c5_noroll.json 2> $O/c5_noroll.err" \
 "timeout -k 10 150 $K --config c5 --accept > $O/c5_roll2.json 2> $O/c5_roll2.err" \
 "timeout -s KILL 150 rocprofv3 --pmc $P1 -d $O/c5_sq1 -o p --output-format csv -- $B5 > $O/c5_sq1.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc $P2 -d $O/c5_sq2 -o p --output-format csv -- $B5 > $O/c5_sq2.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc $P1 -d $O/c3_sq1 -o p --output-format csv -- $B3 > $O/c3_sq1.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc $P2 -d $O/c3_sq2 -o p --output-format csv -- $B3 > $O/c3_sq2.log 2>&1" \
 "timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 > $O/bench_c3.json 2> $O/bench_c3.err" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o c3 --output-format csv -- python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 0 > $O/prof_c3.json 2> $O/prof_c3.log" \
 "timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_c3_fetch -o f --output-format csv -- $B3 > $O/pmc_c3_fetch.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c3_write -o w --output-format csv -- $B3 > $O/pmc_c3_write.log 2>&1"
