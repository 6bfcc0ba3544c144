#!/bin/bash
# Round 4, second call: C5 layout probe (full lane packets, half-mixed row variants) with PMC
# passes; the fetch_ll tree with API fences (DMT_TREE_FENCES build) vs the default on the
# driver's C2 command, interleaved; the new GPU tests (headline kernel vs oracle at full C2,
# service switch, critical_change, TD second-order filter on the device).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04b}
mkdir -p $O
P=scripts/c5_layout_probe
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --calls-iters 0"
FL=build_variants/libdmt_fences.so
PT="python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread"
scripts/gpu_session.sh \
 "timeout -k 10 90 $P 512 10 > $O/probe.jsonl 2> $O/probe.err" \
 "timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o f --output-format csv -- $P 512 2 > $O/pmc_fetch.log 2>&1" \
 "timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o w --output-format csv -- $P 512 2 > $O/pmc_write.log 2>&1" \
 "timeout -k 10 120 $B > $O/c2_def1.json 2> $O/c2_def1.err" \
 "DMT_LIB_PATH=$FL timeout -k 10 120 $B > $O/c2_fen1.json 2> $O/c2_fen1.err" \
 "timeout -k 10 120 $B > $O/c2_def2.json 2> $O/c2_def2.err" \
 "DMT_LIB_PATH=$FL timeout -k 10 120 $B > $O/c2_fen2.json 2> $O/c2_fen2.err" \
 "timeout -k 10 400 $PT tests/test_gpu_parity.py -k 'headline or full_size_sampled' tests/test_deferred.py tests/test_param_update.py tests/test_td_aux.py tests/test_multirank.py > $O/pytest_new.log 2>&1"
