#!/bin/bash
# Round-1 (session c) GPU validation of HEAD: parity tests, smoke, benches (C2 headline, C3,
# C5), rocprofv3 kernel trace of C2, PMC FETCH/WRITE passes (persistent kernel runs 10
# iterations per dispatch: --warmup 10 --steps 10) and the calibration program.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r01c
mkdir -p $O
scripts/gpu_session.sh \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1" \
 "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1" \
 "timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err" \
 "timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err" \
 "timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python bench.py --steps 50 --no-cpu-baseline > $O/prof_c2.log 2>&1" \
 "timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_c2_fetch -o f --output-format csv -- python bench.py --steps 10 --warmup 10 --no-cpu-baseline > $O/pmc_c2_fetch.log 2>&1" \
 "timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c2_write -o w --output-format csv -- python bench.py --steps 10 --warmup 10 --no-cpu-baseline > $O/pmc_c2_write.log 2>&1" \
 "timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_calib_fetch -o f --output-format csv -- scripts/calib_stream > $O/calib_f.log 2>&1" \
 "timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_calib_write -o w --output-format csv -- scripts/calib_stream > $O/calib_w.log 2>&1"
