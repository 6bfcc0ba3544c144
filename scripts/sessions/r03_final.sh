#!/bin/bash
# Round-3 evidence: GPU suite, smoke, the driver's bench command (+ host-phase profile), the
# default bench, rocprofv3 kernel traces (C2 driver command, C3, C5), C2 PMC traffic passes with
# calibration, C2 SQ issue passes, C3/C5 bench lines.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03final}
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64"
B="python bench.py --steps 20 --warmup 20 --no-cpu-baseline --repeats 0 --calls-iters 0"
scripts/gpu_session.sh \
 "timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1" \
 "timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1" \
 "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c2_driver.json 2> $O/bench_c2_driver.err" \
 "DMT_HOST_PROFILE=1 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --calls-iters 0 > $O/bench_c2_hostprof.json 2> $O/bench_c2_hostprof.err" \
 "timeout -k 10 300 python bench.py > $O/bench_c2_default.json 2> $O/bench_c2_default.err" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_c2.json 2> $O/prof_c2.log" \
 "timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_c2_fetch -o f --output-format csv -- $B > $O/pmc_c2_fetch.log 2>&1" \
 "timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c2_write -o w --output-format csv -- $B > $O/pmc_c2_write.log 2>&1" \
 "timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_calib_fetch -o f --output-format csv -- scripts/calib_stream > $O/calib_f.log 2>&1" \
 "timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_calib_write -o w --output-format csv -- scripts/calib_stream > $O/calib_w.log 2>&1" \
 "timeout -s KILL 120 rocprofv3 --pmc $P1 -d $O/sq_p1 -o p --output-format csv -- $B > $O/sq_p1.log 2>&1" \
 "timeout -s KILL 120 rocprofv3 --pmc $P2 -d $O/sq_p2 -o p --output-format csv -- $B > $O/sq_p2.log 2>&1" \
 "timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 > $O/bench_c3.json 2> $O/bench_c3.err" \
 "timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 > $O/bench_c5.json 2> $O/bench_c5.err" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o c3 --output-format csv -- python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 0 > $O/prof_c3.json 2> $O/prof_c3.log" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o c5 --output-format csv -- python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 0 > $O/prof_c5.json 2> $O/prof_c5.log"
