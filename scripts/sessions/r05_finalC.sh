#!/bin/bash
# Round 5, second final tree, part B (C5 on k_block_ps_pk, C3 two chunks ahead): C5 and C3 bench lines, rocprofv3 kernel traces, PMC FETCH/WRITE
# and two SQ passes each; the tutorial (biblock/inference.md) for 1 000 iterations.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05gb}
mkdir -p $O
python scripts/provenance.py > $O/tree.txt
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64"
B5="python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline --calls-iters 0 --repeats 0"
B3="python bench.py --config c3 --steps 4 --warmup 2 --no-cpu-baseline --calls-iters 0 --repeats 0"
scripts/gpu_session.sh \
 "DMT_LANE_SPLIT=0 timeout -k 10 120 python scripts/kbench.py --config c5 --mapping lane --accept --iters 20 > $O/c5_nosplit1.json 2> $O/c5_nosplit1.err" \
 "timeout -k 10 120 python scripts/kbench.py --config c5 --mapping lane --accept --iters 20 > $O/c5_new1.json 2> $O/c5_new1.err" \
 "DMT_LANE_SPLIT=0 timeout -k 10 120 python scripts/kbench.py --config c5 --mapping lane --accept --iters 20 > $O/c5_nosplit2.json 2> $O/c5_nosplit2.err" \
 "timeout -k 10 120 python scripts/kbench.py --config c5 --mapping lane --accept --iters 20 > $O/c5_new2.json 2> $O/c5_new2.err" \
 "timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 > $O/bench_c5.json 2> $O/bench_c5.err" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o c5 --output-format csv -- python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 0 > $O/prof_c5.json 2> $O/prof_c5.log" \
 "timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_c5_fetch -o f --output-format csv -- $B5 > $O/pmc_c5_fetch.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c5_write -o w --output-format csv -- $B5 > $O/pmc_c5_write.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc $P1 -d $O/c5_sq1 -o p --output-format csv -- $B5 > $O/c5_sq1.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc $P2 -d $O/c5_sq2 -o p --output-format csv -- $B5 > $O/c5_sq2.log 2>&1" \
 "timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 > $O/bench_c3.json 2> $O/bench_c3.err" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o c3 --output-format csv -- python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 0 > $O/prof_c3.json 2> $O/prof_c3.log" \
 "timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_c3_fetch -o f --output-format csv -- $B3 > $O/pmc_c3_fetch.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c3_write -o w --output-format csv -- $B3 > $O/pmc_c3_write.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc $P1 -d $O/c3_sq1 -o p --output-format csv -- $B3 > $O/c3_sq1.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc $P2 -d $O/c3_sq2 -o p --output-format csv -- $B3 > $O/c3_sq2.log 2>&1" \
 "timeout -k 10 300 python -u examples/fhn_gamma_inference.py --steps 1000 --burn-in 100 > $O/tutorial.log 2>&1" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_tut -o tut --output-format csv -- python examples/fhn_gamma_inference.py --steps 300 --burn-in 100 > $O/prof_tut.log 2>&1"
