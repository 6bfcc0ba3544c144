#!/bin/bash
# One-hop fetch_ll tail (default) vs the two-hop tail (build_variants/libdmt_twohop.so) on the
# driver's C2 command, interleaved; then the final tree: GPU suite, smoke, bench lines (C2 driver
# command with its CPU leg, default C2, C3, C5), rocprofv3 kernel trace of the driver's command.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03end}
mkdir -p $O
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --calls-iters 0 --repeats 10"
V=DMT_LIB_PATH=build_variants/libdmt_twohop.so
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
scripts/gpu_session.sh \
 "timeout -k 10 300 $PT tests/test_gpu_parity.py -k 'mcmc_run or fetch_ll or c2' > $O/pytest_tail.log 2>&1" \
 "timeout -k 10 200 $B > $O/ab_one1.json 2> $O/ab_one1.err" \
 "$V timeout -k 10 200 $B > $O/ab_two1.json 2> $O/ab_two1.err" \
 "timeout -k 10 200 $B > $O/ab_one2.json 2> $O/ab_one2.err" \
 "$V timeout -k 10 200 $B > $O/ab_two2.json 2> $O/ab_two2.err" \
 "timeout -k 10 900 $PT tests -m gpu > $O/pytest.log 2>&1" \
 "timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1" \
 "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c2_driver.json 2> $O/bench_c2_driver.err" \
 "timeout -k 10 300 python bench.py > $O/bench_c2_default.json 2> $O/bench_c2_default.err" \
 "timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 > $O/bench_c3.json 2> $O/bench_c3.err" \
 "timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 > $O/bench_c5.json 2> $O/bench_c5.err" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_c2.json 2> $O/prof_c2.log"
