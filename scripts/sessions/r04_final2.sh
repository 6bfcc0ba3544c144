#!/bin/bash
# Round 4, last tree: GPU suite + smoke; C2 at the driver's command (with the CPU leg) twice and
# its rocprofv3 kernel trace; C5 bench line, kernel trace, PMC and SQ passes (√dt table build).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04last}
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64"
B5="python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline --calls-iters 0 --repeats 0"
scripts/gpu_session.sh \
 "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1" \
 "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1" \
 "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c2_driver1.json 2> $O/bench_c2_driver1.err" \
 "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c2_driver2.json 2> $O/bench_c2_driver2.err" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --repeats 0 --calls-iters 0 > $O/prof_c2.json 2> $O/prof_c2.log" \
 "timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 > $O/bench_c5.json 2> $O/bench_c5.err" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o c5 --output-format csv -- python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 0 > $O/prof_c5.json 2> $O/prof_c5.log" \
 "timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_c5_fetch -o f --output-format csv -- $B5 > $O/pmc_c5_fetch.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c5_write -o w --output-format csv -- $B5 > $O/pmc_c5_write.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc $P1 -d $O/c5_sq1 -o p --output-format csv -- $B5 > $O/c5_sq1.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc $P2 -d $O/c5_sq2 -o p --output-format csv -- $B5 > $O/c5_sq2.log 2>&1"
