#!/bin/bash
# Round 5, final tree, part A: GPU suite + smoke; C2 at the driver's command twice (with the CPU
# leg); C2 rocprofv3 kernel trace, PMC FETCH/WRITE + calibration, two SQ passes.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05fa}
mkdir -p $O
python scripts/provenance.py > $O/tree.txt
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64"
B2="python bench.py --steps 20 --warmup 20 --no-cpu-baseline --repeats 0 --calls-iters 0"
scripts/gpu_session.sh \
 "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1" \
 "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1" \
 "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c2_driver1.json 2> $O/bench_c2_driver1.err" \
 "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c2_driver2.json 2> $O/bench_c2_driver2.err" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --repeats 0 --calls-iters 0 > $O/prof_c2.json 2> $O/prof_c2.log" \
 "timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_c2_fetch -o f --output-format csv -- $B2 > $O/pmc_c2_fetch.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c2_write -o w --output-format csv -- $B2 > $O/pmc_c2_write.log 2>&1" \
 "timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_calib_fetch -o f --output-format csv -- scripts/calib_stream > $O/pmc_calib_fetch.log 2>&1" \
 "timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_calib_write -o w --output-format csv -- scripts/calib_stream > $O/pmc_calib_write.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc $P1 -d $O/c2_sq1 -o p --output-format csv -- $B2 > $O/c2_sq1.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc $P2 -d $O/c2_sq2 -o p --output-format csv -- $B2 > $O/c2_sq2.log 2>&1"
