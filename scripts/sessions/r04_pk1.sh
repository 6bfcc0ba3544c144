#!/bin/bash
# Round 4: lane packets for fp32 MAP_LANE ensembles — GPU suite, C5 draw timing (packets vs the
# row layout, DMT_PATH_PACKETS=0), C5/C3 bench lines, rocprofv3 kernel stats and PMC passes of C5.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04c}
mkdir -p $O
K="python scripts/kbench.py --mapping lane"
B5="python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline --calls-iters 0 --repeats 0"
scripts/gpu_session.sh \
 "timeout -k 10 200 python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k 'c5 or ragged or lane' > $O/pytest_quick.log 2>&1" \
 "timeout -k 10 150 $K --config c5 --accept > $O/c5_pk.json 2> $O/c5_pk.err" \
 "DMT_PATH_PACKETS=0 timeout -k 10 150 $K --config c5 --accept > $O/c5_row.json 2> $O/c5_row.err" \
 "timeout -k 10 150 $K --config c5 --accept > $O/c5_pk2.json 2> $O/c5_pk2.err" \
 "timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 > $O/bench_c5.json 2> $O/bench_c5.err" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o c5 --output-format csv -- python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 0 > $O/prof_c5.json 2> $O/prof_c5.log" \
 "timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_c5_fetch -o f --output-format csv -- $B5 > $O/pmc_c5_fetch.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c5_write -o w --output-format csv -- $B5 > $O/pmc_c5_write.log 2>&1" \
 "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1"
